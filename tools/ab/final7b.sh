# round-2 final tree: config E (n=4096), config 5 batch, full mode, n=4096 shard emulation
set -o pipefail
O=gpurun_out/final7; mkdir -p $O
timeout -k 10 300 python3 bench.py --config E --steps 2 --warmup 1 --no-cpu --no-interp > $O/bench_E.json 2> $O/bench_E.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_E.json')); print('E', round(d['ms_per_step'],1), d['value'], d.get('phases_ms'))"
timeout -k 10 300 python3 bench.py --config B5 --steps 3 --warmup 1 --no-cpu > $O/bench_B5.json 2> $O/bench_B5.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_B5.json')); print('B5', round(d['ms_per_step'],1), d['value'])"
timeout -k 10 300 python3 bench.py --mode full --steps 5 --warmup 1 --no-cpu --no-interp > $O/bench_full.json 2> $O/bench_full.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_full.json')); print('full', round(d['ms_per_step'],1), d['value'])"
timeout -k 10 300 python3 tools/shard_time.py 4096 2047 --ws 1,2,4,8 --reps 1 > $O/shard_n4096.txt 2>&1 || exit 1
grep -h '"ws"' $O/shard_n4096.txt | cut -c1-90; grep speedup $O/shard_n4096.txt
