#!/bin/bash
# Round 5: config 5's host gap (wall against device span per step), config 4's profile on the
# radix-2^17 tree (its traffic file supersedes r05a_E), and the dealer shards at n=1024 and n=4096.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 python tools/batch_gap.py --steps 6 > $O/batch_gap.txt 2> $O/batch_gap.err || { echo BATCH GAP FAILED; tail -20 $O/batch_gap.err; exit 1; }
cat $O/batch_gap.txt
timeout -k 10 300 python tools/shard_time.py 1024 511 --ws 1,2,4,8 --reps 3 > $O/shard_n1024.txt 2> $O/shard_n1024.err || { echo SHARD 1024 FAILED; tail -20 $O/shard_n1024.err; exit 1; }
cut -c1-160 $O/shard_n1024.txt
timeout -k 10 400 python tools/shard_time.py 4096 2047 --ws 1,2,4,8 --reps 2 > $O/shard_n4096.txt 2> $O/shard_n4096.err || { echo SHARD 4096 FAILED; tail -20 $O/shard_n4096.err; exit 1; }
cut -c1-160 $O/shard_n4096.txt
bash tools/profile.sh r05m_E --config E || { echo PROFILE E FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05m_E --traffic $O/traffic/r05m_E.json --n 4096 --t 2047 --split 4 \
  --split-len 512 > $O/prof_E_summary.txt 2>&1 || { echo SUMMARY E FAILED; tail -20 $O/prof_E_summary.txt; exit 1; }
head -20 $O/prof_E_summary.txt
echo ALL DONE
