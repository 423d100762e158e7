#!/bin/bash
# Round 5: kernel trace of the 8-way n=1024 shard (tools/shard_time.py --ws 8): the device timeline of
# one shard call (busy time per kernel, idle gaps).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r05r2
mkdir -p $O
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/shard_time.py --ws 8 --reps 3 > $O/shard.log 2>&1) \
  || { echo TRACE FAILED; tail -20 $O/shard.log; exit 1; }
tail -2 $O/shard.log | cut -c1-200
f=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/shard_timeline.py $f --gap-ms 0.2 > $O/timeline.txt 2>&1; cat $O/timeline.txt
echo ALL DONE
