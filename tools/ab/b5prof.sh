# kernel stats of config 5 (10,000 x n=64 ceremonies)
set -o pipefail
mkdir -p gpurun_out/b5prof
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/b5prof/trace" -o run -- python3 $REPO/bench.py --config B5 --steps 1 --warmup 1 --no-cpu --no-interp > "$REPO/gpurun_out/b5prof/log.txt" 2>&1
