#!/bin/bash
# Round 5: radix-2^15 combs as the default and the batch outcome kept on the device (one host
# round trip per batch): the whole GPU suite, then radix 2^15 (default) against 2^11 / 2^16 / 2^17
# builds on config 5 and the headline.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
A=$R/ab_build
bash tools/ab/ab.sh r05g_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "r15=" \
  "r16=DKG_AMD_LIB=$A/r16/libdkg_amd.so" "r17=DKG_AMD_LIB=$A/r17/libdkg_amd.so" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05g_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05g_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "r15=" \
  "r11=DKG_AMD_LIB=$A/r11/libdkg_amd.so" "r16=DKG_AMD_LIB=$A/r16/libdkg_amd.so" "r17=DKG_AMD_LIB=$A/r17/libdkg_amd.so" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05g_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
