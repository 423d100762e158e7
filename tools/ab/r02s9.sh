# schedule knobs on the final kernels: dealer-chunk streams 1..4 (n=1024 default line)
set -o pipefail
O=gpurun_out/s9; mkdir -p $O
for k in 2 3 4 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --streams $k > $O/b_s$k.json 2> $O/b_s$k.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_s$k.json')); print('streams $k', round(d['ms_per_step'],2))"
done
