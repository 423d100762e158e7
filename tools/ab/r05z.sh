#!/bin/bash
# Round 5: the N > 1 line's counter lower bound (the one-GPU INT64 share): the gloo rehearsal tests.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05z
mkdir -p $O/lines
DKG_SAVE_LINES=$O/lines timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bench_dist.py > $O/t_dist.log 2>&1 \
  || { echo DIST FAILED; tail -30 $O/t_dist.log; exit 1; }
tail -1 $O/t_dist.log
echo ALL DONE
