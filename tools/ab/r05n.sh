#!/bin/bash
# Round 5: config 5's outcomes through pinned staging -- the batch tests, the host gap per step, the line.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py -k "batch" \
  > $O/t_batch.log 2>&1 || { echo BATCH TESTS FAILED; tail -30 $O/t_batch.log; exit 1; }
tail -1 $O/t_batch.log
timeout -k 10 300 python tools/batch_gap.py --steps 6 > $O/batch_gap.txt 2> $O/batch_gap.err || { echo BATCH GAP FAILED; tail -20 $O/batch_gap.err; exit 1; }
cat $O/batch_gap.txt
timeout -k 10 300 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-200 $O/bench_B5.json
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05n/bench_B5.json").read().strip().splitlines()[-1])
print("B5 wall", round(d["ms_per_step"], 2), "device", d["phases_ms"])
PY
echo ALL DONE
