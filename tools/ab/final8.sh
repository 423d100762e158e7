# round-2 evidence on the final tree: rocprof trace + PMC passes, default bench line, shard timings, gloo rehearsal
set -o pipefail
O=gpurun_out/final8; mkdir -p $O
tools/profile.sh r02v8 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r02v8 gpurun_out/prof_r02v8/traffic.json 1024 511 4 128 > gpurun_out/prof_r02v8/summary.txt || exit 1
head -12 gpurun_out/prof_r02v8/summary.txt
cp gpurun_out/prof_r02v8/traffic.json profiles/r02_pmc_traffic.json
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['ms_per_step'],2), d['value'], d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline']['traffic'], d['cpu_baseline']['value'], d['interp_mode']['ms_per_step'], d['stepping_redos'])"
timeout -k 10 200 python3 tools/shard_time.py 1024 511 --ws 1,2,4,8 --reps 5 > $O/shard_n1024.txt 2>&1 || exit 1
grep speedup $O/shard_n1024.txt
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/gloo2.txt 2> $O/gloo2.err || exit 1
tail -1 $O/gloo2.txt | cut -c1-300
