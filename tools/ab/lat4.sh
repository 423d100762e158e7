# refresh the secondary bench lines and the n=4096 shard table after the short multipliers
set -o pipefail
mkdir -p gpurun_out/lat4
timeout -k 10 300 python3 tools/shard_time.py 4096 2047 --ws 1,2,4,8 --reps 1 > gpurun_out/lat4/shard4096.txt 2>&1 || exit 1
grep -h '"ws"\|speedup' gpurun_out/lat4/shard4096.txt | cut -c1-200
timeout -k 10 300 python3 bench.py --config E --steps 2 --warmup 1 --no-interp > gpurun_out/lat4/E.json 2> gpurun_out/lat4/E.err || exit 1
timeout -k 10 300 python3 bench.py --mode full --steps 10 --warmup 2 --no-interp > gpurun_out/lat4/full.json 2> gpurun_out/lat4/full.err || exit 1
timeout -k 10 300 python3 bench.py --config B5 --steps 5 --warmup 1 --no-interp > gpurun_out/lat4/B5.json 2> gpurun_out/lat4/B5.err || exit 1
for f in E full B5; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), d['value'], d['config'].get('degree_split'), d['config'].get('recombination'), d.get('phases_ms'))" gpurun_out/lat4/$f.json; done
