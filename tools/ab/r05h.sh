#!/bin/bash
# Round 5: radix-2^17 combs and the lazy-reduction share evaluation -- the whole GPU suite, then the
# round's bench lines (headline with its CPU baseline, config 5, full mode, config 4).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-200 $O/bench_D.json
timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-200 $O/bench_B5.json
timeout -k 10 300 python bench.py --mode full > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FULL FAILED; tail -20 $O/bench_full.err; exit 1; }
cut -c1-200 $O/bench_full.json
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-200 $O/bench_E.json
echo ALL DONE
