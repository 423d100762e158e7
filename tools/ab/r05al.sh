#!/bin/bash
# Round 5: dkg_shard_prepare_device -- the sharded finalise's outcome-independent half (final and public
# shares, the terms' decode) on the side stream beside the combine -- plus the finalise's pinned
# staging: the shard / distributed GPU tests, then the steps after the shard on one GPU
# (tools/exchange_time.py, world-size-1 RCCL group) with and without the prepare step, three rounds of 25 runs
# each (the per-run wall time after the shard's device span: median and min).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05al
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_dist.py \
  tests/test_gpu_bench_dist.py -k "shard or dist or gloo" > $O/t_shard.log 2>&1 || { echo SHARD TESTS FAILED; tail -30 $O/t_shard.log; exit 1; }
tail -1 $O/t_shard.log
bash tools/ab/ab.sh r05al_ex 3 300 "python tools/exchange_time.py --reps 25" "prep=" "noprep=DKG_SHARD_PREPARE=0" \
  || { echo AB FAILED; exit 1; }
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05al_ex/*.out")):
    for l in open(f):
        if l.startswith("{"):
            j = json.loads(l)
            print(f.split("/")[-1], j["exchange_and_combine_ms"], j["after_shard_ms_median"], j["after_shard_ms_min"])
PY
echo ALL DONE
