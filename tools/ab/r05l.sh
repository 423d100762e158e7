#!/bin/bash
# Round 5, final: the whole GPU suite and smoke() of the round's tree, then the round's bench lines
# (headline, config 5, full mode, config 4) with CPU baselines, and full mode's profile.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-200 $O/bench_D.json
timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-200 $O/bench_B5.json
timeout -k 10 300 python bench.py --mode full > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FULL FAILED; tail -20 $O/bench_full.err; exit 1; }
cut -c1-200 $O/bench_full.json
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-200 $O/bench_E.json
bash tools/profile.sh r05l_full --mode full || { echo PROFILE FULL FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05l_full --traffic $O/traffic/r05l_full.json --n 1024 --t 511 --split 4 \
  --split-len 128 --mode full > $O/prof_full_summary.txt 2>&1 || { echo SUMMARY FULL FAILED; exit 1; }
echo ALL DONE
