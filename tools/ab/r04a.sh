set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py -k "binomial_schedules or stepping_modes or stepping_tail or config5 or stepping_formulas or full_mode or hybrid or faults or batch or interp_mode_goldens or finalise" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in "" "--binomial 3" "--stepping 3" "--binomial 3 --stepping 3"; do
  timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu $v > $O/b5_$(echo $v | tr -d ' -').json 2>$O/b5_err.log || { echo BENCH FAILED $v; tail -20 $O/b5_err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],1), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/b5_$(echo $v | tr -d ' -').json "$v"
done
for v in "" "--binomial 3"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-interp $v > $O/d_$(echo $v | tr -d ' -').json 2>$O/d_err.log || { echo BENCH FAILED; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/d_$(echo $v | tr -d ' -').json "$v"
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode full > $O/full.json 2>$O/full_err.log || { echo FULL BENCH FAILED; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('full', round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/full.json
for lib in "" "ab_build/c9/libdkg_amd.so"; do
  for cfg in "D" "B5"; do
    DKG_AMD_LIB=${lib:-dkg_amd/libdkg_amd.so} timeout -k 10 300 python bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-interp > $O/comb_${cfg}_$(basename $(dirname ${lib:-x/base})).json 2>$O/comb_err.log || { echo COMB BENCH FAILED; tail -5 $O/comb_err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('comb', sys.argv[1], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/comb_${cfg}_$(basename $(dirname ${lib:-x/base})).json
  done
done
