# full-rate limb doubling (fe_dbl): full GPU tests and the default bench line
set -o pipefail
O=gpurun_out/s14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 > $O/b$i.json 2> $O/b$i.err || exit 1
python3 -c "import json; d=json.load(open('$O/b$i.json')); k=d['roofline']['all_kernels']; print(round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
