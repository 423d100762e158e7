# per-wave binomial (k_binom_wave) on the GPU: parity of every schedule, then config-5 A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_scale.py -k "binomial_schedules or stepping_tail or config5 or batch_verify" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
for b in 0 3; do
  timeout -k 10 300 python bench.py --config B5 --steps 3 --warmup 1 --no-cpu --binomial $b > $O/b5_b${b}_$i.json 2>$O/err.log || { echo BENCH FAILED; tail -5 $O/err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],1), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/b5_b${b}_$i.json
done
done
for lib in dkg_amd/libdkg_amd.so ab_build/dec/libdkg_amd.so dkg_amd/libdkg_amd.so ab_build/dec/libdkg_amd.so; do
  tag=$(basename $(dirname $lib))
  DKG_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode full > $O/full_${tag}.json 2>$O/err.log || { echo FULL FAILED; tail -5 $O/err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],2), d['roofline']['all_kernels']['dec_mul']['ms_per_pass'])" $O/full_${tag}.json
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 $R/bench.py --config B5 --steps 1 --warmup 0 --no-cpu --streams 1 > $O/pf.log 2>&1 || { echo PMC FAILED; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 $R/bench.py --config B5 --steps 1 --warmup 0 --no-cpu --streams 1 > $O/pw.log 2>&1 || { echo PMC FAILED; exit 1; }
echo done
cd $R
for lib in dkg_amd/libdkg_amd.so ab_build/c11/libdkg_amd.so; do
  for cfg in D B5; do
    tag=$(basename $(dirname $lib))
    DKG_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-interp > $O/comb_${cfg}_${tag}.json 2>$O/err.log || { echo COMB FAILED; tail -5 $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()}, d['phases_ms'])" $O/comb_${cfg}_${tag}.json
  done
done
