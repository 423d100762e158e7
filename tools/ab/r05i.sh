#!/bin/bash
# Round 5: profiles of the round's tree (headline and config 5: kernel trace + SQ / FETCH / WRITE /
# VALU passes, traffic files), and the 2/4/8-way n=1024 shard with five short pieces against four.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "full_mode or hybrid or member_keys" \
  > $O/t_full.log 2>&1 || { echo FULL TESTS FAILED; tail -30 $O/t_full.log; exit 1; }
tail -1 $O/t_full.log
A=$R/ab_build
bash tools/ab/ab.sh r05i_full 2 300 "python bench.py --mode full --steps 5 --warmup 1 --no-cpu" "k10=" \
  "k8=DKG_AMD_LIB=$A/k8/libdkg_amd.so" "k12=DKG_AMD_LIB=$A/k12/libdkg_amd.so" || { echo AB FULL FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05i_full > $O/ab_full.txt 2>&1; cat $O/ab_full.txt
bash tools/profile.sh r05i_D || { echo PROFILE D FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05i_D --traffic $O/traffic/r05i_D.json --n 1024 --t 511 --split 4 \
  --split-len 128 > $O/prof_D_summary.txt 2>&1 || { echo SUMMARY D FAILED; tail -5 $O/prof_D_summary.txt; exit 1; }
head -12 $O/prof_D_summary.txt
bash tools/profile.sh r05i_B5 --config B5 || { echo PROFILE B5 FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05i_B5 --traffic $O/traffic/r05i_B5.json --n 64 --t 31 --split 1 \
  --split-len 32 --batch 10000 > $O/prof_B5_summary.txt 2>&1 || { echo SUMMARY B5 FAILED; tail -5 $O/prof_B5_summary.txt; exit 1; }
head -12 $O/prof_B5_summary.txt
bash tools/ab/ab.sh r05i_shard 2 300 "python tools/shard_time.py --ws 2,4,8 --reps 3" "u4=--split 4" "u5=--split 5" \
  || { echo AB SHARD FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05i_shard > $O/ab_shard.txt 2>&1; cat $O/ab_shard.txt
bash tools/ab/ab.sh r05i_E 2 300 "python bench.py --config E --steps 2 --warmup 1 --no-cpu --no-interp" "u4=--split 4" "u5=--split 5" \
  || { echo AB E FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05i_E > $O/ab_E.txt 2>&1; cat $O/ab_E.txt
echo ALL DONE
