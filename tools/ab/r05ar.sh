#!/bin/bash
# Round 5, final tree: the driver's round-end steps rehearsed -- GPU suite, smoke(), the default bench
# line (N=1 with its CPU baseline) and the 2-rank gloo line on one GPU.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ar
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-200 $O/bench_D.json
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo BENCH GLOO2 FAILED; tail -20 $O/bench_gloo2.err; exit 1; }
cut -c1-200 $O/bench_gloo2.json
echo ALL DONE
