# dedicated stepping additions: full GPU tests, then bench A/B of the stepping formulas + kernel trace
set -o pipefail
O=gpurun_out/s8; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for f in 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --step-formula $f > $O/b_f$f.json 2> $O/b_f$f.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_f$f.json')); k=d['roofline']['all_kernels']; print('formula $f', round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$O/tr" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 > "$REPO/$O/tr.log" 2>&1) || exit 1
python3 - $O <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f"{sys.argv[1]}/tr/run_kernel_stats.csv"))}
print({k[:34]: (c, round(x)) for k, (c, x) in rows.items() if "affine" in k or "combine" in k or "stepping" in k})
PY
