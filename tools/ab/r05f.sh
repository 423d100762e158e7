#!/bin/bash
# Round 5: comb radix 2^15 / 2^16 / 2^17 on config 5 and the headline; five short pieces against four
# on the 2/4/8-way n=1024 shards; a kernel trace of the real (two-stream)
# config-5 schedule at radix 2^15 for its host gaps.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05f
mkdir -p $O
A=$R/ab_build
bash tools/ab/ab.sh r05f_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" \
  "r15=DKG_AMD_LIB=$A/r15/libdkg_amd.so" "r16=DKG_AMD_LIB=$A/r16/libdkg_amd.so" "r17=DKG_AMD_LIB=$A/r17/libdkg_amd.so" \
  || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05f_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05f_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" \
  "r15=DKG_AMD_LIB=$A/r15/libdkg_amd.so" "r16=DKG_AMD_LIB=$A/r16/libdkg_amd.so" "r17=DKG_AMD_LIB=$A/r17/libdkg_amd.so" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05f_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
bash tools/ab/ab.sh r05f_shard 2 300 "python tools/shard_time.py --ws 2,4,8 --reps 3" "u4=--split 4" "u5=--split 5" \
  || { echo AB SHARD FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05f_shard > $O/ab_shard.txt 2>&1; cat $O/ab_shard.txt
export TMPDIR=/tmp
DKG_AMD_LIB=$A/r15/libdkg_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_b5 -o run \
  -- python3 bench.py --config B5 --steps 2 --warmup 1 --no-cpu > $O/trace_b5.log 2>&1 || { echo TRACE FAILED; tail -5 $O/trace_b5.log; exit 1; }
echo ALL DONE
