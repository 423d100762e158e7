#!/bin/bash
# Round 5: the per-step binomial's rerun guard with its word copied into pinned memory ahead of the
# callers' own sync (no round trip of its own): the redo test and the GPU suite, then the headline
# (two rounds) and the 8-way shard (three) against -DDKG_BINOM_STEP_DED=0 (prev), interleaved.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05ag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
P="prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so"
bash tools/ab/ab.sh r05ag_shard 3 300 "python tools/shard_time.py --ws 8 --reps 3" "new=" "$P" || { echo AB SHARD FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05ag_shard > $O/ab_shard.txt 2>&1; cat $O/ab_shard.txt
bash tools/ab/ab.sh r05ag_d 2 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "$P" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05ag_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
echo ALL DONE
