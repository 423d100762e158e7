# k_affine_pieces block size 4 (current) vs 2 vs 8: kernel trace of the serialised pass + bench
set -o pipefail
O=gpurun_out/s15; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
for v in cur blk2 blk8 cur blk2; do
  lib=$REPO/dkg_amd/libdkg_amd.so; [ $v != cur ] && lib=$REPO/ab_build/$v/libdkg_amd.so
  (cd /tmp && DKG_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$O/tr_$v" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 > "$REPO/$O/tr_$v.log" 2>&1) || exit 1
  DKG_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 - $O $v <<'PY'
import csv, json, sys
O, v = sys.argv[1:3]
d = json.load(open(f"{O}/b_{v}.json"))
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f"{O}/tr_{v}/run_kernel_stats.csv"))}
print(v, round(d["ms_per_step"], 2), {k[:24]: round(x) for k, x in rows.items() if "affine" in k or "combine" in k})
PY
done
