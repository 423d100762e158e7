# short-multiplier recombination: dealer-shard timings per forced split, and n=4096 (config E)
set -o pipefail
mkdir -p gpurun_out/lat2
for cfg in "--split 3" "--split 4" "--split 4 --stepping 2" "--split 5" "--split 3 --combine 1"; do
  tag=$(echo $cfg | tr -d ' -')
  echo "== $cfg"
  timeout -k 10 240 python3 tools/shard_time.py --ws 1,2,4,8 --reps 5 $cfg > gpurun_out/lat2/s_$tag.txt 2>&1 || exit 1
  python3 -c "import json,sys; [print(d['ws'], d['ms_wall'], d['split'], d['split_len'], d['combine']) for d in map(json.loads, open(sys.argv[1])) if 'ws' in d]" gpurun_out/lat2/s_$tag.txt
done
for cfg in "--combine 0" "--combine 1"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python3 bench.py --config E --steps 1 --warmup 1 --no-cpu --no-interp $cfg > gpurun_out/lat2/E_$tag.json 2> gpurun_out/lat2/E_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']['all_kernels']; print('E', sys.argv[2], round(d['ms_per_step'],1), d['config']['degree_split'], {k:(v['ms_per_pass'], round(v['frac'],3)) for k,v in r.items()})" gpurun_out/lat2/E_$tag.json "$cfg"
done
