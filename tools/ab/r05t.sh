#!/bin/bash
# Round 5: the single-ceremony drivers' outcomes on the device with one host round trip (as the
# batches): the GPU suite, then the headline and full mode against the previous library, two
# interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab/ab.sh r05t_d 2 300 "python bench.py --steps 10 --warmup 2 --no-cpu --no-interp" "new=" "prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05t_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05t_d/*.out")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "wall", round(d["ms_per_step"], 3), "phases", d["phases_ms"])
PY
echo ALL DONE
