#!/bin/bash
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/r05ao
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ao/trace -o run -- \
  python3 $R/tools/shard_time.py --ws 8 --reps 2 > $R/gpurun_out/r05ao/trace.log 2>&1 || { echo TRACE FAILED; tail -20 $R/gpurun_out/r05ao/trace.log; exit 1; }
cd $R
f=$(find gpurun_out/r05ao/trace -name "*kernel_trace.csv" | head -1); echo $f
python tools/shard_timeline.py $f > gpurun_out/r05ao/timeline.txt 2>&1; head -12 gpurun_out/r05ao/timeline.txt
