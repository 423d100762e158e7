#!/bin/bash
# Round 5: the per-step binomial's steps without lane pairs with dedicated additions, the verification
# rerun with the complete formula when a group was marked: the redo test on the product library (green)
# and without the rerun (ab_build/norerun: red), the GPU suite, then the headline, config 4 and
# the 8-way shard against -DDKG_BINOM_STEP_DED=0 (prev), two interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05af
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k "binomial_dedicated_redo" \
  > $O/t_redo.log 2>&1 || { echo REDO TEST FAILED; tail -30 $O/t_redo.log; exit 1; }
tail -1 $O/t_redo.log
DKG_AMD_LIB=$R/ab_build/norerun/libdkg_amd.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gpu.py -k "binomial_dedicated_redo" > $O/t_norerun.log 2>&1
rc=$?; echo "without the rerun: rc=$rc (expected nonzero)"; tail -3 $O/t_norerun.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
P="prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so"
bash tools/ab/ab.sh r05af_d 2 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "$P" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05af_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
bash tools/ab/ab.sh r05af_shard 2 300 "python tools/shard_time.py --ws 8 --reps 3" "new=" "$P" || { echo AB SHARD FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05af_shard > $O/ab_shard.txt 2>&1; cat $O/ab_shard.txt
bash tools/ab/ab.sh r05af_e 1 400 "python bench.py --config E --steps 2 --warmup 1 --no-cpu --no-interp" "new=" "$P" || { echo AB E FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05af_e > $O/ab_e.txt 2>&1; cat $O/ab_e.txt
python - <<'PY'
import glob, json
for d in ("ab_r05af_d", "ab_r05af_e"):
    for f in sorted(glob.glob(f"gpurun_out/{d}/*.out")):
        j = json.loads(open(f).read().strip().splitlines()[-1])
        k = j["roofline"]["all_kernels"]
        print(d, f.split("/")[-1], "wall", round(j["ms_per_step"], 2), {x: k[x]["ms_per_pass"] for x in k})
PY
echo ALL DONE
