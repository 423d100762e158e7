#!/bin/bash
# Round 5, second GPU call: packed decision bitmaps (the sharded exchange), the prefetching per-wave
# binomial (mode 5) on the goldens and an interleaved config-5 A/B against mode 0, then config 4's
# bench line with its first traffic file (profiles/pmc_traffic/r05a_E.json) and the headline line.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05b
mkdir -p $O
DKG_SAVE_LINES=$O timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_pack.py tests/test_gpu_dist.py tests/test_gpu_bench_dist.py tests/test_gpu.py tests/test_gpu_scale.py \
  -k "pack or dist or multi_rank or binomial_schedules or config5 or sharded or shard_combine" \
  > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/ab/ab.sh r05b_pf 2 300 "python bench.py --config B5 --steps 3 --warmup 1 --no-cpu" "m0=--binomial 0" "m5=--binomial 5" \
  || { echo AB FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05b_pf > $O/ab_pf.txt 2>&1; cat $O/ab_pf.txt
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err \
  || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-300 $O/bench_E.json
timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-300 $O/bench_D.json
echo ALL DONE
