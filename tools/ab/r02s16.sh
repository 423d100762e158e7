# tiled position-major placement: full GPU tests, kernel trace, bench
set -o pipefail
O=gpurun_out/s16; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$O/tr" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 > "$REPO/$O/tr.log" 2>&1) || exit 1
python3 - $O <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f"{sys.argv[1]}/tr/run_kernel_stats.csv"))}
print({k[:24]: v for k, v in rows.items() if "place" in k or "commit" in k})
PY
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 > $O/b$i.json 2> $O/b$i.err || exit 1
python3 -c "import json; d=json.load(open('$O/b$i.json')); print(round(d['ms_per_step'],2), d['phases_ms'])"
done
