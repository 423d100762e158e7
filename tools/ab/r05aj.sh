#!/bin/bash
# Round 5: dkg_shard_finalise_device's small host transfers (qualified in, decode flags and mpk out)
# through pinned staging instead of pageable bounces: the sharded steps after the shard on one GPU
# (tools/exchange_time.py, world-size-1 RCCL group) against the previous library, three rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "shard" \
  > $O/t_shard.log 2>&1 || { echo SHARD TESTS FAILED; tail -30 $O/t_shard.log; exit 1; }
tail -1 $O/t_shard.log
bash tools/ab/ab.sh r05aj_ex 3 300 "python tools/exchange_time.py --reps 5" "new=" "prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so" \
  || { echo AB FAILED; exit 1; }
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05aj_ex/*.out")):
    for l in open(f):
        if l.startswith("{"):
            j = json.loads(l)
            print(f.split("/")[-1], j["exchange_and_combine_ms"], j["parts_ms"])
PY
echo ALL DONE
