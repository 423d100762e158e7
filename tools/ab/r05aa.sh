#!/bin/bash
# Round 5: the per-wave binomial with dedicated additions and a complete redo of the marked column
# groups (config 5): the GPU suite (forced per-wave schedules on the fault fixtures take the redo),
# then config 5 against -DDKG_BINOM_WAVE_DED=0 (prev), two interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab/ab.sh r05aa_b5 2 300 "python bench.py --config B5 --steps 4 --warmup 1 --no-cpu" "new=" "prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so" \
  || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05aa_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05aa_b5/*.out")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    k = j["roofline"]["all_kernels"]
    print(f.split("/")[-1], "wall", round(j["ms_per_step"], 2), "device", j["phases_ms"]["total"], {x: k[x]["ms_per_pass"] for x in k})
PY
echo ALL DONE
