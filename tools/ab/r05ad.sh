#!/bin/bash
# Round 5, final tree (dedicated per-wave binomial): GPU suite and smoke, then the headline and config 5
# each profiled (kernel trace + SQ / FETCH / WRITE / VALU passes, traffic) together with its bench line
# on the same box, and full mode's line.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ad
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile.sh r05ad_D || { echo PROFILE D FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05ad_D --traffic $O/traffic/r05ad_D.json --n 1024 --t 511 --split 4 \
  --split-len 128 > $O/prof_D_summary.txt 2>&1 || { echo SUMMARY D FAILED; tail -5 $O/prof_D_summary.txt; exit 1; }
head -5 $O/prof_D_summary.txt
DKG_PMC_TRAFFIC_DIR=$O/traffic timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-150 $O/bench_D.json
bash tools/profile.sh r05ad_B5 --config B5 || { echo PROFILE B5 FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05ad_B5 --traffic $O/traffic/r05ad_B5.json --n 64 --t 31 --split 1 \
  --split-len 32 --batch 10000 > $O/prof_B5_summary.txt 2>&1 || { echo SUMMARY B5 FAILED; tail -5 $O/prof_B5_summary.txt; exit 1; }
head -5 $O/prof_B5_summary.txt
DKG_PMC_TRAFFIC_DIR=$O/traffic timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-150 $O/bench_B5.json
timeout -k 10 300 python bench.py --mode full > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FULL FAILED; tail -20 $O/bench_full.err; exit 1; }
cut -c1-150 $O/bench_full.json
echo ALL DONE
