#!/bin/bash
# Round 5: the fixed-base comb's entry prefetch (PF) and the occupancy of the fixed-base kernels
# (min waves per SIMD W: 4 = 128 VGPRs with spills, 3 = 168, 2 = 256) on config 5 and the headline.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05j
mkdir -p $O
A=$R/ab_build
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu.py -k "fixed_base or share_gen or ceremony_honest or ceremony_faults or batch_verify or batch_device or full_mode_verify or random_ceremonies" \
  > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/ab/ab.sh r05j_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "pf1w4=" \
  "pf1w3=DKG_AMD_LIB=$A/pf1w3/libdkg_amd.so" "pf1w2=DKG_AMD_LIB=$A/pf1w2/libdkg_amd.so" \
  "pf0w4=DKG_AMD_LIB=$A/pf0w4/libdkg_amd.so" "pf0w3=DKG_AMD_LIB=$A/pf0w3/libdkg_amd.so" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05j_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05j_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "pf1w4=" \
  "pf1w3=DKG_AMD_LIB=$A/pf1w3/libdkg_amd.so" "pf0w4=DKG_AMD_LIB=$A/pf0w4/libdkg_amd.so" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05j_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
