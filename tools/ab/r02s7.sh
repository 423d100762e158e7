# 8-way n=1024 shard: per-phase breakdown at U = 4 (short) and U = 5, 6, 8 (powers); 4-way for reference
set -o pipefail
O=gpurun_out/s7; mkdir -p $O
for sp in 4 5 6 8; do
  timeout -k 10 120 python3 tools/shard_time.py 1024 511 --ws 8 --reps 5 --streams 1 --split $sp > $O/ws8_s1_u$sp.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/shard_time.py 1024 511 --ws 8 --reps 5 --split $sp > $O/ws8_u$sp.txt 2>&1 || exit 1
  echo "U=$sp"; head -1 $O/ws8_s1_u$sp.txt | cut -c1-400; head -1 $O/ws8_u$sp.txt | cut -c1-120
done
