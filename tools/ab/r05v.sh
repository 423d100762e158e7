#!/bin/bash
# Round 5: a single ceremony's round-1 commitments deferred into the verification's chunks (as the
# batches): the GPU suite, then the headline against -DDKG_R1_DEFER=0 (prev), three interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab/ab.sh r05v_d 3 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05v_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05v_d/*.out")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "wall", round(j["ms_per_step"], 2), j["phases_ms"])
PY
echo ALL DONE
