# coalesced affine normalisation: targeted tests, kernel trace, bench A/B of the addend modes
set -o pipefail
O=gpurun_out/s6; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "combine or recombination or headline or n1024 or n4096 or n1100" > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$O/tr" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 > "$REPO/$O/tr.log" 2>&1) || exit 1
python3 - $O <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f"{sys.argv[1]}/tr/run_kernel_stats.csv"))}
print({k[:28]: round(x) for k, x in rows.items() if "affine" in k or "combine" in k or "stepping" in k})
PY
for a in 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --addends $a > $O/b_a$a.json 2> $O/b_a$a.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_a$a.json')); print('addends $a', round(d['ms_per_step'],2))"
done
