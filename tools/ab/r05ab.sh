#!/bin/bash
# Round 5: the dedicated binomial's redo test -- green on the product library, and red on a build
# without the redo launch (ab_build/noredo: the test must catch a skipped redo).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "binomial_dedicated_redo or binomial_schedules" \
  > $O/t_redo.log 2>&1 || { echo REDO TEST FAILED; tail -30 $O/t_redo.log; exit 1; }
tail -1 $O/t_redo.log
DKG_AMD_LIB=$R/ab_build/noredo/libdkg_amd.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gpu.py -k "binomial_dedicated_redo" > $O/t_noredo.log 2>&1
rc=$?; echo "without the redo launch: rc=$rc (expected nonzero)"
tail -3 $O/t_noredo.log
echo ALL DONE
