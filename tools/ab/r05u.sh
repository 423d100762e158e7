#!/bin/bash
# Round 5: (wl) the stepping's one-wave segments exchange without workgroup barriers; (new) + the
# fixed-base kernels fetch each comb entry by LDS-DMA one window ahead.  The GPU suite of the new
# tree, then config 5 (prev / wl / new), the headline and full mode (prev / new), two rounds each.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
P="prev=DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so"
bash tools/ab/ab.sh r05u_b5 2 300 "python bench.py --config B5 --steps 4 --warmup 1 --no-cpu" "new=" "$P" \
  "wl=DKG_AMD_LIB=$R/ab_build/wl/libdkg_amd.so" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05u_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05u_d 2 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "$P" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05u_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
bash tools/ab/ab.sh r05u_full 2 300 "python bench.py --mode full --steps 5 --warmup 1 --no-cpu" "new=" "$P" || { echo AB FULL FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05u_full > $O/ab_full.txt 2>&1; cat $O/ab_full.txt
python - <<'PY'
import glob, json
for d in ("ab_r05u_b5", "ab_r05u_d", "ab_r05u_full"):
    for f in sorted(glob.glob(f"gpurun_out/{d}/*.out")):
        j = json.loads(open(f).read().strip().splitlines()[-1])
        k = j["roofline"]["all_kernels"]
        print(d, f.split("/")[-1], "wall", round(j["ms_per_step"], 2), {x: k[x]["ms_per_pass"] for x in k})
PY
echo ALL DONE
