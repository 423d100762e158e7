#!/bin/bash
# Round 5, final tree (dedicated per-step binomial with its rerun guard): GPU suite and smoke, then the
# headline profiled (kernel trace + SQ / FETCH / WRITE / VALU passes, traffic) together with its bench
# line on the same box, and full mode's line (config 5's binomial is per-wave: r05ah/r05ae stand).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ah
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile.sh r05ah_D || { echo PROFILE D FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05ah_D --traffic $O/traffic/r05ah_D.json --n 1024 --t 511 --split 4 \
  --split-len 128 > $O/prof_D_summary.txt 2>&1 || { echo SUMMARY D FAILED; tail -5 $O/prof_D_summary.txt; exit 1; }
head -5 $O/prof_D_summary.txt
DKG_PMC_TRAFFIC_DIR=$O/traffic timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-150 $O/bench_D.json
timeout -k 10 300 python bench.py --mode full > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FULL FAILED; tail -20 $O/bench_full.err; exit 1; }
cut -c1-150 $O/bench_full.json
echo ALL DONE
