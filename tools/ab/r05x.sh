#!/bin/bash
# Round 5: chunk-stream count for config 5 (2 default, 3, 4) and the headline (2, 3), two interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05x
mkdir -p $O
bash tools/ab/ab.sh r05x_b5 2 300 "python bench.py --config B5 --steps 4 --warmup 1 --no-cpu" "s2=--streams 2" "s3=--streams 3" "s4=--streams 4" \
  || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05x_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05x_d 2 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "s2=--streams 2" "s3=--streams 3" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05x_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
