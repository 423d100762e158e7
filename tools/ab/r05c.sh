#!/bin/bash
# Round 5, third GPU call: the n=1024 unsplit repack test that went silent in r05b (alone, then after
# the config-5 batch, with a 150-s per-test timeout that dumps the stacks), the split-comb check and
# the rest of r05b (config-5 binomial prefetch A/B, config-4 and headline lines).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread --durations=0 \
  "tests/test_gpu_scale.py::test_stepping_tail_repack_unsplit_n1024" \
  > $O/t_unsplit.log 2>&1 || { echo UNSPLIT FAILED; tail -60 $O/t_unsplit.log; exit 1; }
grep -E "passed|failed|s call" $O/t_unsplit.log | head -5
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread --durations=0 \
  tests/test_gpu_scale.py -k "config5_full or stepping_tail" > $O/t_c5.log 2>&1 || { echo C5+UNSPLIT FAILED; tail -60 $O/t_c5.log; exit 1; }
grep -E "passed|failed|s call" $O/t_c5.log | head -8
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu.py -k "check_split or binomial_schedules" \
  > $O/t_check.log 2>&1 || { echo CHECK TESTS FAILED; tail -40 $O/t_check.log; exit 1; }
tail -2 $O/t_check.log
bash tools/ab/ab.sh r05c_b5 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "m0=--binomial 0" "m5=--binomial 5" "c1=--check 1" \
  || { echo AB FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05c_b5 > $O/ab_b5.txt 2>&1; cat $O/ab_b5.txt
bash tools/ab/ab.sh r05c_d 2 300 "python bench.py --steps 5 --warmup 1 --no-cpu --no-interp" "c0=--check 0" "c1=--check 1" \
  || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05c_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err \
  || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-300 $O/bench_E.json
echo ALL DONE
