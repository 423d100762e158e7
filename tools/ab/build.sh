#!/bin/bash
# A/B builds of the HIP library with an alternative fe25519.h (field arithmetic variant).
#   tools/ab/build.sh <variant-header> <name>  ->  ab_build/<name>/libdkg_amd.so
# Load a variant with DKG_AMD_LIB=ab_build/<name>/libdkg_amd.so (dkg_amd/_lib.py).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
hdr=$(readlink -f "$1"); name=$2
dst=$ROOT/ab_build/$name
rm -rf "$dst"; mkdir -p "$dst" "$ROOT/ab_build/include"
cp "$ROOT/include/dkg_amd.h" "$ROOT/ab_build/include/"
cp -r "$ROOT/dkg_amd/csrc" "$ROOT/dkg_amd/Makefile" "$dst/"
cp "$hdr" "$dst/csrc/fe25519.h"
make -s -j8 -C "$dst" HDR="$(echo "$dst"/csrc/*.h)"
echo "$dst/libdkg_amd.so"
