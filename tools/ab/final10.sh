# final tree: config E (n=4096) and config 5 (10,000 x n=64) lines
set -o pipefail
O=gpurun_out/final10; mkdir -p $O
timeout -k 10 300 python3 bench.py --config E --steps 2 --warmup 1 --no-cpu --no-interp > $O/bench_E.json 2> $O/bench_E.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_E.json')); print('E', round(d['ms_per_step'],1), d['value'], {a: b['ms_per_pass'] for a, b in d['roofline']['all_kernels'].items()})"
timeout -k 10 300 python3 bench.py --config B5 --steps 3 --warmup 1 --no-cpu > $O/bench_B5.json 2> $O/bench_B5.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_B5.json')); print('B5', round(d['ms_per_step'],1), d['value'])"
