#!/bin/bash
# Round 5: the shard's qualification on the device, its master-key terms and shares on the side stream
# (no host round trip inside the shard call): the sharded / multi-device GPU tests, then the 1/2/4/8-way
# n=1024 shards against the previous library (ab_build/prev), two interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_multi.py \
  tests/test_gpu_bench_dist.py tests/test_gpu_scale.py -k "shard or rank or multi or dist or bench" > $O/t_shard.log 2>&1 \
  || { echo SHARD TESTS FAILED; tail -30 $O/t_shard.log; exit 1; }
tail -1 $O/t_shard.log
bash tools/ab/ab.sh r05s2 2 300 "python tools/shard_time.py --ws 1,2,4,8 --reps 3" "new=" "prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so" \
  || { echo AB FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05s2 > $O/ab.txt 2>&1; cat $O/ab.txt
echo ALL DONE
