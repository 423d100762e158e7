#!/bin/bash
# A/B builds of the HIP library: a copy of dkg_amd/csrc with some files replaced and/or extra
# compiler flags, built into ab_build/<name>/libdkg_amd.so (load it with DKG_AMD_LIB=<that path>,
# e.g. as a tools/ab/ab.sh variant).
#   tools/ab/build.sh <name> [csrc-file=replacement-path ...] [-DFLAG ...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; shift
dst=$ROOT/ab_build/$name
rm -rf "$dst"; mkdir -p "$dst" "$ROOT/ab_build/include"
cp "$ROOT/include/dkg_amd.h" "$ROOT/ab_build/include/"
cp -r "$ROOT/dkg_amd/csrc" "$ROOT/dkg_amd/Makefile" "$dst/"
extra=""
for a in "$@"; do
  case $a in
    -D*) extra="$extra $a" ;;
    *=*) cp "$(readlink -f "${a#*=}")" "$dst/csrc/${a%%=*}" ;;
    *) echo "unknown argument $a" >&2; exit 2 ;;
  esac
done
make -s -j8 -C "$dst" FLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-result$extra"
echo "$dst/libdkg_amd.so"
