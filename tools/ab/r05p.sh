#!/bin/bash
# Round 5: the outcome helpers split into device and host halves (one round trip in the sharded
# combine): the GPU suite, then the sharded run's steps after the shard (pack, all-gathers, combine,
# finalise, copy-out) on one GPU over a world-size-1 RCCL group.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo GPU SUITE FAILED; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python tools/exchange_time.py --reps 5 > $O/exchange_n1024.txt 2> $O/exchange_n1024.err || { echo EXCHANGE FAILED; tail -20 $O/exchange_n1024.err; exit 1; }
tail -1 $O/exchange_n1024.txt
echo ALL DONE
