# cheapest-chain lattice rows: GPU tests + default bench (no CPU baseline) twice
set -o pipefail
mkdir -p gpurun_out/lat5
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lat5/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/lat5/pytest.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 > gpurun_out/lat5/b$i.json 2> gpurun_out/lat5/b$i.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']['all_kernels']; print(round(d['ms_per_step'],2), d['config']['degree_split'], {k:(v['ms_per_pass'], round(v['frac'],3)) for k,v in r.items()}, d['roofline']['traffic'])" gpurun_out/lat5/b$i.json
done
timeout -k 10 240 python3 tools/shard_time.py --ws 8 --reps 5 > gpurun_out/lat5/s8.txt 2>&1 || exit 1
grep '"ws"' gpurun_out/lat5/s8.txt | cut -c1-120
