#!/bin/bash
# Round 5, final tree: the GPU suite and smoke(), the round's bench lines (headline, config 5, full
# mode, config 4) with CPU baselines, the N > 1 rehearsal lines (2 and 3 gloo ranks on one GPU), the
# dealer shards at 1/2/4/8 ranks and the steps after the shard.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_D.json 2> $O/bench_D.err || { echo BENCH D FAILED; tail -20 $O/bench_D.err; exit 1; }
cut -c1-150 $O/bench_D.json
timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-150 $O/bench_B5.json
timeout -k 10 300 python bench.py --mode full > $O/bench_full.json 2> $O/bench_full.err || { echo BENCH FULL FAILED; tail -20 $O/bench_full.err; exit 1; }
cut -c1-150 $O/bench_full.json
timeout -k 10 400 python bench.py --config E --steps 3 --warmup 1 --no-interp > $O/bench_E.json 2> $O/bench_E.err || { echo BENCH E FAILED; tail -20 $O/bench_E.err; exit 1; }
cut -c1-150 $O/bench_E.json
mkdir -p $O/lines
DKG_SAVE_LINES=$O/lines timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bench_dist.py > $O/t_dist.log 2>&1 \
  || { echo DIST LINES FAILED; tail -30 $O/t_dist.log; exit 1; }
tail -1 $O/t_dist.log
timeout -k 10 300 python tools/shard_time.py --ws 1,2,4,8 --reps 3 > $O/shard_n1024.txt 2> $O/shard.err || { echo SHARD FAILED; tail -20 $O/shard.err; exit 1; }
tail -1 $O/shard_n1024.txt
timeout -k 10 300 python tools/exchange_time.py --reps 5 > $O/exchange.txt 2> $O/exchange.err || { echo EXCHANGE FAILED; tail -20 $O/exchange.err; exit 1; }
tail -1 $O/exchange.txt
echo ALL DONE
