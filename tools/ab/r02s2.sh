# session-2 check: GPU tests, then the default bench line
set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s2/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/s2/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/s2/bench.json')); print(round(d['ms_per_step'],2), d['value'], d['roofline']['kernel'], round(d['roofline']['frac'],3), d.get('phase_ms') or '', d['interp_mode']['ms_per_step'])"
