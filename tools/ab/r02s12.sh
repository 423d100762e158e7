# width-3 NAF on the first recombination scalar: targeted tests, bench A/B (addends 0 vs 2), trace
set -o pipefail
O=gpurun_out/s12; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "combine or recombination or headline or n1024 or n4096 or spot" > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for a in 0 2 0 2; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --addends $a > $O/b_a$a.json 2> $O/b_a$a.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_a$a.json')); k=d['roofline']['all_kernels']; print('addends $a', round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
