# deferred round-1 commitments in the batch (BatchRound1): batch parity, then config-5 A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py -k "batch or config5 or stepping_tail or binomial_schedules" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in "" "--no-overlap"; do
    tag=b5$(echo $v | tr -d ' -')_$i
    timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu $v > $O/$tag.json 2>$O/err.log || { echo BENCH FAILED; tail -5 $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],1), d['phases_ms'])" $O/$tag.json $tag
  done
  DKG_AMD_LIB=$R/ab_build/prev/libdkg_amd.so timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu > $O/b5prev_$i.json 2>$O/err.log || { echo BENCH FAILED; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('prev', round(d['ms_per_step'],1), d['phases_ms'])" $O/b5prev_$i.json
done
cd $R
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/gloo2.json 2>$O/gloo2.err || { echo GLOO FAILED; tail -20 $O/gloo2.err; exit 1; }
cat $O/gloo2.json | cut -c1-600
for f in 0 2 0 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --no-interp --field $f > $O/d_field$f.json 2>$O/err.log || { echo FIELD FAILED; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('field', sys.argv[2], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/d_field$f.json $f
done
