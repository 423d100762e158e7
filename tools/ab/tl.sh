# kernel timeline of the default (2 chunk streams) ceremony
set -o pipefail
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$REPO/gpurun_out/tl/trace" -o run -- python3 $REPO/bench.py --no-cpu --no-interp --steps 2 --warmup 1 > "$REPO/gpurun_out/tl/log.txt" 2>&1
