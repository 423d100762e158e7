#!/bin/bash
# Round 5: the tail-state race fix (one state layout for every repack phase) on the n=1024 unsplit
# test (twice) and config 5 at full size; the per-wave binomial back on k_to_column_major; then A/Bs
# of the comb radix (2^11 default vs 2^13 / 2^14 / 2^15 builds) and of the binomial's column-major
# last step (cm1) on config 5, and the radix on the headline and full mode.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread \
  tests/test_gpu_scale.py -k "stepping_tail or config5_full" > $O/t_tail.log 2>&1 \
  || { echo TAIL TESTS FAILED; grep -E "PASS|FAIL|Error|assert" $O/t_tail.log | head -30; exit 1; }
grep -E "passed|failed" $O/t_tail.log | tail -2
timeout -k 10 300 python -u tools/dbg_unsplit.py --identity 1 > $O/dbg_id1.txt 2>&1 || { echo DBG FAILED; tail -20 $O/dbg_id1.txt; exit 1; }
grep -c '"dec2_diffs": 0, ' $O/dbg_id1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu.py \
  -k "binomial_schedules or check_split or batch" > $O/t_gpu.log 2>&1 || { echo GPU TESTS FAILED; tail -30 $O/t_gpu.log; exit 1; }
tail -1 $O/t_gpu.log
A=$R/ab_build
bash tools/ab/ab.sh r05e_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "r11=" \
  "cm1=DKG_AMD_LIB=$A/cm1/libdkg_amd.so" "r13=DKG_AMD_LIB=$A/r13/libdkg_amd.so" "r14=DKG_AMD_LIB=$A/r14/libdkg_amd.so" \
  "r15=DKG_AMD_LIB=$A/r15/libdkg_amd.so" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05e_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05e_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "r11=" \
  "r13=DKG_AMD_LIB=$A/r13/libdkg_amd.so" "r15=DKG_AMD_LIB=$A/r15/libdkg_amd.so" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05e_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
bash tools/ab/ab.sh r05e_full 2 300 "python bench.py --mode full --steps 5 --warmup 1 --no-cpu" "r11=" \
  "r13=DKG_AMD_LIB=$A/r13/libdkg_amd.so" "r15=DKG_AMD_LIB=$A/r15/libdkg_amd.so" || { echo AB FULL FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05e_full > $O/ab_full.txt 2>&1; cat $O/ab_full.txt
echo ALL DONE
