# round-2 evidence on the final tree: GPU tests, rocprof trace + PMC passes, default bench line, 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/final6
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final6/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/final6/pytest.txt; [ $rc -eq 0 ] || exit $rc
tools/profile.sh r02v6 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r02v6 gpurun_out/prof_r02v6/traffic.json 1024 511 4 128 > gpurun_out/prof_r02v6/summary.txt || exit 1
head -8 gpurun_out/prof_r02v6/summary.txt
timeout -k 10 300 python3 bench.py > gpurun_out/final6/bench.json 2> gpurun_out/final6/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/final6/bench.json')); print(round(d['ms_per_step'],2), d['value'], d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline']['traffic'], d['cpu_baseline']['value'], d['interp_mode']['ms_per_step'])"
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > gpurun_out/final6/gloo2.txt 2> gpurun_out/final6/gloo2.err || exit 1
tail -1 gpurun_out/final6/gloo2.txt | cut -c1-300
