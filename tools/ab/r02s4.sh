# A/B on one box: stepping truncation (lib variants), affine vs projective addends (kernel traces)
set -o pipefail
O=gpurun_out/s4; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
for v in cur notrunc cur notrunc; do
  lib=$REPO/dkg_amd/libdkg_amd.so; [ $v = notrunc ] && lib=$REPO/ab_build/notrunc/libdkg_amd.so
  DKG_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 --addends 1 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); k=d['roofline']['all_kernels']; print('$v', round(d['ms_per_step'],2), {a: b['ms_per_pass'] for a, b in k.items()})"
done
for a in 0 1; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$O/trace_a$a" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 --addends $a > "$REPO/$O/trace_a$a.log" 2>&1) || exit 1
  f=$(find $O/trace_a$a -name "*kernel_stats.csv" | head -1); echo "== addends $a"; cut -d, -f1-4 $f | head -12
done
