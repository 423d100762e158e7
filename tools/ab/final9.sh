# final tree: default bench line (with CPU baseline and interpolation-mode side line)
set -o pipefail
O=gpurun_out/final9; mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['ms_per_step'],2), d['value'], d['roofline']['kernel'], round(d['roofline']['frac'],3), d['cpu_baseline']['value'], {a: (b['ms_per_pass'], round(b['frac'],3)) for a, b in d['roofline']['all_kernels'].items()})"
