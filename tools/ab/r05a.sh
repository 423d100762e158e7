#!/bin/bash
# Round 5, first GPU call: the N > 1 bench line on one GPU
# (2 and 3 gloo ranks), the flag-layout fix at n=1024 unsplit, the multi-device context's tests and
# timing tool, then config 4's first profile and the round's bench lines of configs 4, 3 and 5.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05a
mkdir -p $O
DKG_SAVE_LINES=$O timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_bench_dist.py tests/test_gpu_multi.py tests/test_gpu_scale.py -k "stepping_tail or multi" \
  > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/multi_time.py --devices 0,0 --reps 3 > $O/multi_time.txt 2> $O/multi_time.err \
  || { echo MULTI_TIME FAILED; tail -20 $O/multi_time.err; exit 1; }
cat $O/multi_time.txt
bash tools/profile.sh r05a_E --config E || { echo PROFILE FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_r05a_E --traffic $O/traffic/r05a_E.json --n 4096 --t 2047 --split 4 \
  --split-len 512 > $O/prof_E_summary.txt 2>&1 || { echo PMC SUMMARY FAILED; tail -20 $O/prof_E_summary.txt; exit 1; }
head -30 $O/prof_E_summary.txt
DKG_PMC_TRAFFIC_DIR=$O/traffic timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp \
  > $O/bench_E.json 2> $O/bench_E.err || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-300 $O/bench_E.json
timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-300 $O/bench_D.json
timeout -k 10 400 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err \
  || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-300 $O/bench_B5.json
echo ALL DONE
