#!/bin/bash
# Round 5: the per-step binomial's launch thresholds re-tuned with its dedicated additions on: lane
# pairs below DKG_BINOM_PAIR_WAVES (1.0: 0.75, 1.5) and the column-sum copy below DKG_BINOM_ILP_WAVES
# (1.5: 1.0, 2.5) waves per SIMD, on the 8-way and 2-way n=1024 shards (three rounds) and the
# headline (one), interleaved.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aq
mkdir -p $O
V=("new=")
for v in p075 p15 i10 i25; do V+=("$v=DKG_AMD_LIB=$R/ab_build/$v/libdkg_amd.so"); done
bash tools/ab/ab.sh r05aq_ws8 3 300 "python tools/shard_time.py --ws 8 --reps 3" "${V[@]}" || { echo AB WS8 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05aq_ws8 > $O/ab_ws8.txt 2>&1; cat $O/ab_ws8.txt
bash tools/ab/ab.sh r05aq_ws2 2 300 "python tools/shard_time.py --ws 2 --reps 3" "${V[@]}" || { echo AB WS2 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05aq_ws2 > $O/ab_ws2.txt 2>&1; cat $O/ab_ws2.txt
bash tools/ab/ab.sh r05aq_d 1 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "${V[@]}" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05aq_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
