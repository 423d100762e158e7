# A/B: decryption table slices (capped 16,384 waves vs one launch) and the mixed binomial order
# on config 5 (kernel trace + FETCH_SIZE per variant)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04b
mkdir -p $O
for i in 1 2; do
  for lib in dkg_amd/libdkg_amd.so ab_build/dec/libdkg_amd.so; do
    tag=$(basename $(dirname $lib))
    DKG_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode full > $O/full_${tag}_$i.json 2>$O/err.log || { echo FULL FAILED; tail -5 $O/err.log; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],2), d['roofline']['all_kernels']['dec_mul']['ms_per_pass'])" $O/full_${tag}_$i.json
  done
done
export TMPDIR=/tmp
cd /tmp
for b in 0 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_b$b -o run -- python3 $R/bench.py --config B5 --steps 1 --warmup 0 --no-cpu --streams 1 --binomial $b > $O/tr_b$b.log 2>&1 || { echo TRACE FAILED; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_b$b -o run -- python3 $R/bench.py --config B5 --steps 1 --warmup 0 --no-cpu --streams 1 --binomial $b > $O/pf_b$b.log 2>&1 || { echo PMC FAILED; exit 1; }
done
echo done
