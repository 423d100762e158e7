# two positions per lane in the dedicated stepping: targeted tests, bench A/B (formula 0 vs 2), trace
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stepping or combine or headline or n1024 or n4096 or n1100 or golden or spot" > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for f in 0 2 0 2; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --step-formula $f > $O/b_f$f.json 2> $O/b_f$f.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_f$f.json')); k=d['roofline']['all_kernels']; print('formula $f', round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
timeout -k 10 200 python3 tools/shard_time.py 1024 511 --ws 1,8 --reps 5 > $O/shard.txt 2>&1 || exit 1
grep -h ms_wall $O/shard.txt | cut -c1-120
