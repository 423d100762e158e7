# kernel traces of the 8-way n=1024 shard (tools/shard_time.py --ws 8) under binomial modes $@
set -e -o pipefail
export TMPDIR=/tmp
R=$(pwd)
for b in "$@"; do
  mkdir -p gpurun_out/trs_b$b
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trs_b$b -o run -- python3 $R/tools/shard_time.py --ws 8 --reps 2 --binomial $b > $R/gpurun_out/trs_b$b/log.txt 2>&1)
done
