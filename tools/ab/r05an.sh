#!/bin/bash
# Round 5: the stepping's dedicated pass with lane pairs (k_stepping_pair) for whole-column launches
# at <= 2 waves per SIMD (the 8-way n=1024 shard): its redo test and the shard tests, the GPU suite,
# a kernel trace of the 8-way shard, then the 8-way and 4-way shards (four / two rounds) and the
# headline (one) against -DDKG_STEP_PAIR=0 (prev), interleaved.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05an
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py \
  -k "pair_stepping or shard_ranks_n1024" > $O/t_pair.log 2>&1 || { echo PAIR TESTS FAILED; tail -30 $O/t_pair.log; exit 1; }
tail -1 $O/t_pair.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05an/trace -o run -- \
  python3 $R/tools/shard_time.py --ws 8 --reps 2 > $O/trace.log 2>&1 || { echo TRACE FAILED; tail -20 $O/trace.log; exit 1; }
cd $R
python tools/shard_timeline.py $(find gpurun_out/r05an/trace -name "*kernel_trace.csv" | head -1) > $O/timeline.txt 2>&1; head -8 $O/timeline.txt
P="prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so"
bash tools/ab/ab.sh r05an_ws8 4 300 "python tools/shard_time.py --ws 8 --reps 3" "new=" "$P" || { echo AB WS8 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05an_ws8 > $O/ab_ws8.txt 2>&1; cat $O/ab_ws8.txt
bash tools/ab/ab.sh r05an_ws4 2 300 "python tools/shard_time.py --ws 4 --reps 3" "new=" "$P" || { echo AB WS4 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05an_ws4 > $O/ab_ws4.txt 2>&1; cat $O/ab_ws4.txt
bash tools/ab/ab.sh r05an_d 1 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "$P" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05an_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
