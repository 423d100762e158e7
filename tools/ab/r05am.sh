#!/bin/bash
# Round 5: dkg_ctx_binomial_reruns -- the crafted-identity redo test asserts that only the dedicated
# per-step schedule reruns (ceremony and dealer-shard entry points) and that honest broadcasts and
# honest ragged ceremonies never do; then the whole GPU suite and smoke().
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05am
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py \
  -k "binomial_dedicated_redo or honest_ragged" > $O/t_rerun.log 2>&1 || { echo RERUN TESTS FAILED; tail -30 $O/t_rerun.log; exit 1; }
tail -1 $O/t_rerun.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ALL DONE
