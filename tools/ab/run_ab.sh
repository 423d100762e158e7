#!/bin/bash
# GPU side of the fe_mul A/B (run from the repo root on the GPU box):
# per variant, bench.py at config D (n=1024, t=511) and a kernel trace of the serialised ceremony.
#   tools/ab/run_ab.sh <tag> <name>=<lib.so> ...
set -e -o pipefail
TAG=$1; shift
REPO=$(pwd)
OUT=$REPO/gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}; lib=$(readlink -f "${spec#*=}")
  DKG_AMD_LIB=$lib timeout -k 10 240 python3 bench.py --no-cpu --steps 10 --warmup 2 > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  cat "$OUT/bench_$name.json"
  (cd /tmp && DKG_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --streams 1 --steps 2 --warmup 1 > "$OUT/trace_$name.log" 2>&1)
done
echo done
