# round-2 evidence after the short-multiplier recombination (U=4 by the cost model at n=1024)
set -o pipefail
mkdir -p gpurun_out/lat3
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lat3/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/lat3/pytest.txt; [ $rc -eq 0 ] || exit $rc
tools/profile.sh r02v5 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r02v5 gpurun_out/prof_r02v5/traffic.json 1024 511 4 128 > gpurun_out/prof_r02v5/summary.txt || exit 1
head -16 gpurun_out/prof_r02v5/summary.txt
timeout -k 10 300 python3 bench.py > gpurun_out/lat3/bench.json 2> gpurun_out/lat3/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/lat3/bench.json')); print(round(d['ms_per_step'],2), d['value'], d['config']['degree_split'], d['config']['recombination'], d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline']['traffic'], d['cpu_baseline']['value'])"
