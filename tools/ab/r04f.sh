# Round-4 final: the whole GPU suite and smoke on HEAD, then the bench lines (with the CPU baseline)
# of the headline, config 4, config 5 and full mode
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() {  # tag args...
  tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>$O/$tag.err || { echo BENCH FAILED $tag; tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d['value'], d['roofline']['frac'], d['roofline'].get('traffic'), d['cpu_baseline']['value'])" $O/$tag.json $tag
}
line D
line E --config E --steps 2 --warmup 1
line B5 --config B5 --steps 3 --warmup 1
line full --mode full
