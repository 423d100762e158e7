#!/bin/bash
# Round 5: config 4 profiled on the final tree (dedicated per-step binomial with its rerun guard), with
# its bench line on the same box so that the rocprof averages and the line's HIP-event times agree.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ai
mkdir -p $O
bash tools/profile.sh r05ai_E --config E || { echo PROFILE E FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05ai_E --traffic $O/traffic/r05ai_E.json --n 4096 --t 2047 --split 4 \
  --split-len 512 > $O/prof_E_summary.txt 2>&1 || { echo SUMMARY E FAILED; tail -20 $O/prof_E_summary.txt; exit 1; }
head -6 $O/prof_E_summary.txt
DKG_PMC_TRAFFIC_DIR=$O/traffic timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-150 $O/bench_E.json
echo ALL DONE
