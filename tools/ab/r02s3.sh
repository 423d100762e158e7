# affine addends: targeted GPU tests, then bench A/B of the addend modes on one box
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "combine or recombination or headline or n1024 or n4096 or n1100" > gpurun_out/s3/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/s3/pytest.txt; [ $rc -eq 0 ] || exit $rc
for a in 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --addends $a > gpurun_out/s3/bench_a$a.json 2> gpurun_out/s3/bench_a$a.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/s3/bench_a$a.json')); print('addends $a', round(d['ms_per_step'],2), d['phases_ms'])"
done
