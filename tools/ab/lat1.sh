set -o pipefail
mkdir -p gpurun_out/lat1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lat1/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/lat1/pytest.txt; [ $rc -eq 0 ] || exit $rc
for cfg in "--split 3 --combine 0" "--split 3 --combine 1" "--split 4 --combine 0" "--split 2 --combine 0" "--split 0 --combine 0"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 10 --warmup 2 $cfg > gpurun_out/lat1/b_$tag.json 2> gpurun_out/lat1/b_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']['all_kernels']; print(sys.argv[2], round(d['ms_per_step'],2), d['config']['degree_split'], d['config'].get('recombination'), {k:(v['ms_per_pass'], round(v['frac'],3)) for k,v in r.items()})" gpurun_out/lat1/b_$tag.json "$cfg"
done
