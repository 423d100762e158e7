# binomial position pairs: targeted tests, bench A/B over the pairing threshold, 8-way shard
set -o pipefail
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pairing or recombination or headline or n1024 or n1100 or spot" > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for p in 0 2 4 8 0 2 4 8; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --binom-pair $p > $O/b_p$p.json 2> $O/b_p$p.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_p$p.json')); k=d['roofline']['all_kernels']; print('pair $p', round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
