#!/bin/bash
# Round 5: staggered chunk streams (DKG_CHUNK_STAGGER = the binomial step of chunk 0 at which chunk 1
# starts) on the headline, two interleaved rounds; config 5 (per-wave binomial: chunk 1 after chunk
# 0's binomial) once.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05o
mkdir -p $O
bash tools/ab/ab.sh r05o_d 2 300 "python bench.py --steps 10 --warmup 2 --no-cpu --no-interp" "s0=" \
  "s16=DKG_CHUNK_STAGGER=16" "s48=DKG_CHUNK_STAGGER=48" "s96=DKG_CHUNK_STAGGER=96" "s127=DKG_CHUNK_STAGGER=127" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05o_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
bash tools/ab/ab.sh r05o_b5 1 300 "python bench.py --config B5 --steps 4 --warmup 1 --no-cpu" "s0=" "s1=DKG_CHUNK_STAGGER=1" \
  || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05o_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
echo ALL DONE
