# HEAD (radix-2^11 combs, per-wave binomial with register carry, 32k-wave decryption slices):
# the whole GPU suite, then A/Bs on config 5, the headline and full mode
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  DKG_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu --no-interp "$@" > $O/$tag.json 2>$O/err.log || { echo BENCH FAILED $tag; tail -5 $O/err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k:v['ms_per_pass'] for k,v in d['roofline']['all_kernels'].items()})" $O/$tag.json $tag
}
for i in 1 2; do
  run b5_head_$i dkg_amd/libdkg_amd.so --config B5 --steps 3 --warmup 1
  run b5_nocarry_$i ab_build/nocarry/libdkg_amd.so --config B5 --steps 3 --warmup 1
  run b5_perstep_$i dkg_amd/libdkg_amd.so --config B5 --steps 3 --warmup 1 --binomial 3
done
for i in 1 2; do
  run d_head_$i dkg_amd/libdkg_amd.so --steps 10 --warmup 2
  run d_c10_$i ab_build/c10/libdkg_amd.so --steps 10 --warmup 2
done
run full_head dkg_amd/libdkg_amd.so --steps 5 --warmup 1 --mode full
run full_c10 ab_build/c10/libdkg_amd.so --steps 5 --warmup 1 --mode full
