#!/bin/bash
# Round 5: diagnosis of the n=1024 unsplit repack mismatch, then the rest of r05c (config-5 test at
# full size, split-comb check tests, config-5 A/Bs of the binomial prefetch, the split-comb check and
# the comb radix 2^12 / 2^13 builds; headline A/B of the split check; config-4 line).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05d
mkdir -p $O
timeout -k 10 200 python -u tools/dbg_unsplit.py --identity 1 > $O/dbg_id1.txt 2>&1 || { echo DBG1 FAILED; tail -20 $O/dbg_id1.txt; exit 1; }
cat $O/dbg_id1.txt
timeout -k 10 200 python -u tools/dbg_unsplit.py --identity 0 > $O/dbg_id0.txt 2>&1 || { echo DBG0 FAILED; tail -20 $O/dbg_id0.txt; exit 1; }
cat $O/dbg_id0.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py \
  -k "check_split or config5_full" > $O/t_check.log 2>&1 || { echo CHECK TESTS FAILED; tail -40 $O/t_check.log; exit 1; }
tail -2 $O/t_check.log
bash tools/ab/ab.sh r05d_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "m0=--binomial 0" "m5=--binomial 5" "c1=--check 1" \
  "r12=DKG_AMD_LIB=$R/ab_build/c12/libdkg_amd.so --binomial 0" "r13=DKG_AMD_LIB=$R/ab_build/c13/libdkg_amd.so --binomial 0" \
  || { echo AB FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05d_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05d_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "c0=--check 0" "c1=--check 1" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05d_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err \
  || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-300 $O/bench_E.json
echo ALL DONE
