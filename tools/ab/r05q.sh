#!/bin/bash
# Round 5: host-side latency of the synchronous calls -- the runtime's blocking stream wait against
# polling (DKG_SPIN_SYNC=1): the headline (wall over device span), the sharded run's steps after the
# shard (tools/exchange_time.py, fused all-gather), config 5; then the multi-GPU tests of the new exchange.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05q
mkdir -p $O
for v in 0 1; do
  DKG_SPIN_SYNC=$v timeout -k 10 300 python tools/exchange_time.py --reps 5 > $O/exchange_s$v.txt 2> $O/exchange_s$v.err || { echo EXCHANGE $v FAILED; tail -20 $O/exchange_s$v.err; exit 1; }
  echo "spin=$v $(tail -1 $O/exchange_s$v.txt)"
done
bash tools/ab/ab.sh r05q_d 2 300 "python bench.py --steps 10 --warmup 2 --no-cpu --no-interp" "s0=" "s1=DKG_SPIN_SYNC=1" || { echo AB D FAILED; exit 1; }
python tools/ab/summary.py gpurun_out/ab_r05q_d > $O/ab_d.txt 2>&1; cat $O/ab_d.txt
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_r05q_d/*.out")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "wall", round(d["ms_per_step"], 3), "device total", d["phases_ms"]["total"])
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_bench_dist.py tests/test_gpu_pack.py \
  > $O/t_dist.log 2>&1 || { echo DIST TESTS FAILED; tail -30 $O/t_dist.log; exit 1; }
tail -1 $O/t_dist.log
echo ALL DONE
