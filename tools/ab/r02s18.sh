# share evaluation beside the verification: side-stream grid cap 0 (uncapped) / 256 / 512 / 1024
set -o pipefail
O=gpurun_out/s18; mkdir -p $O
REPO=$(pwd)
for v in sb0 cur sb256 sb1024 sb0 cur sb256 sb1024; do
  lib=$REPO/dkg_amd/libdkg_amd.so; [ $v != cur ] && lib=$REPO/ab_build/$v/libdkg_amd.so
  DKG_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --no-interp --steps 20 --warmup 2 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', round(d['ms_per_step'],2), d['phases_ms'])"
done
