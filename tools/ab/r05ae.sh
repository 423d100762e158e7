#!/bin/bash
# Round 5: config 5's line against the corrected traffic file (pmc_traffic/r05ad_B5.json: the redo
# launches of the dedicated per-wave binomial kept apart from its pass).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ae
mkdir -p $O
timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-150 $O/bench_B5.json
echo ALL DONE
