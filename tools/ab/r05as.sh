#!/bin/bash
# Round 5: the fixed-base comb loop with the next window's entry loaded before this window's addition
# (-DDKG_COMB_PREFETCH=1: more spills -- k_commit_pm 92 -> 212 B, k_check_both<0> 20 -> 168 B per lane)
# against the plain loop on config 5 and the headline, two interleaved rounds.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05as
mkdir -p $O
P="pf=DKG_AMD_LIB=$R/ab_build/pf/libdkg_amd.so"
bash tools/ab/ab.sh r05as_b5 2 300 "python bench.py --config B5 --steps 4 --warmup 1 --no-cpu" "new=" "$P" || { echo AB B5 FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05as_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05as_d 2 300 "python bench.py --steps 8 --warmup 2 --no-cpu --no-interp" "new=" "$P" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05as_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
python - <<'PY'
import glob, json
for d in ("ab_r05as_b5", "ab_r05as_d"):
    for f in sorted(glob.glob(f"gpurun_out/{d}/*.out")):
        j = json.loads(open(f).read().strip().splitlines()[-1])
        k = j["roofline"]["all_kernels"]
        print(d, f.split("/")[-1], round(j["ms_per_step"], 2), {x: k[x]["ms_per_pass"] for x in k})
PY
echo ALL DONE
