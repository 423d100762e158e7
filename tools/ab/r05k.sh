#!/bin/bash
# Round 5: occupancy of the fixed-base kernels (min waves per SIMD 4 / 3 / 2) on config 5 and the
# headline, without the comb prefetch.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05k
mkdir -p $O
A=$R/ab_build
bash tools/ab/ab.sh r05k_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "w4=" \
  "w3=DKG_AMD_LIB=$A/w3/libdkg_amd.so" "w2=DKG_AMD_LIB=$A/w2/libdkg_amd.so" \
  "bw2=DKG_AMD_LIB=$A/bw2/libdkg_amd.so" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05k_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05k_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "w4=" \
  "w3=DKG_AMD_LIB=$A/w3/libdkg_amd.so" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05k_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
