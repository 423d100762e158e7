# kernel timeline of the default ceremony (2 chunk streams): the first milliseconds
set -o pipefail
O=gpurun_out/s17; mkdir -p $O
REPO=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$REPO/$O/tr" -o run -- python3 "$REPO/bench.py" --no-cpu --no-interp --steps 2 --warmup 1 > "$REPO/$O/tr.log" 2>&1) || exit 1
ls $O/tr
