# HEAD parity on the paths changed since r04d (deferred batch commitments, per-wave binomial writing
# the column-major table, five-piece short multipliers), then config-5 and headline A/Bs
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04e
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu.py tests/test_gpu_scale.py -k "multi or batch or config5 or stepping_tail or binomial_schedules or combine_modes or split or recombination_modes or faults_baseline" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "" "--no-overlap"; do
  tag=b5$(echo $v | tr -d ' -')
  timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu $v > $O/$tag.json 2>$O/err.log || { echo BENCH FAILED; tail -5 $O/err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],1), d['phases_ms'], {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/$tag.json $tag
done
DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu > $O/b5prev.json 2>$O/err.log || { echo BENCH FAILED; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('prev', round(d['ms_per_step'],1), d['phases_ms'])" $O/b5prev.json
for s in 4 5 4 5; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --no-interp --split $s > $O/d_split$s.json 2>$O/err.log || { echo SPLIT FAILED; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('split', sys.argv[2], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/d_split$s.json $s
done
for s in 4 5; do
  timeout -k 10 300 python tools/shard_time.py --ws 4,8 --reps 3 --split $s > $O/shard_split$s.txt 2>$O/err.log || { echo SHARD FAILED; exit 1; }
  tail -3 $O/shard_split$s.txt | cut -c1-300
done
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/gloo2.json 2>$O/gloo2.err || { echo GLOO FAILED; tail -20 $O/gloo2.err; exit 1; }
cut -c1-400 $O/gloo2.json
