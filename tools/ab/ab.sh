#!/bin/bash
# A/B harness (run on the GPU box from the repo root): one command under several variants,
# interleaved over R rounds so that box drift hits every variant alike.
#   tools/ab/ab.sh <tag> <rounds> <timeout_s> "<command>" "<name>=<extra args>" ...
# Each run is `<command> <extra args>` under its own `timeout -k 10 <timeout_s>`; stdout goes to
# gpurun_out/ab_<tag>/<name>.<round>.out (stderr .err).  A variant may also select a library build:
# "<name>=DKG_AMD_LIB=<path> <extra args>" (dkg_amd/_lib.py honours DKG_AMD_LIB; tools/ab/build.sh), or set
# any DKG_* runtime knob ("<name>=DKG_CHUNK_STAGGER=64").
# Stops at the first failing run.  Summary: tools/ab/summary.py gpurun_out/ab_<tag>.
set -e -o pipefail
TAG=$1; ROUNDS=$2; TMO=$3; CMD=$4; shift 4
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
for ((r = 0; r < ROUNDS; r++)); do
  for spec in "$@"; do
    name=${spec%%=*}; extra=${spec#*=}
    envs=(); args=()
    for w in $extra; do
      if [[ $w == DKG_*=* ]]; then envs+=("$w"); else args+=("$w"); fi
    done
    env "${envs[@]}" timeout -k 10 "$TMO" $CMD "${args[@]}" > "$OUT/$name.$r.out" 2> "$OUT/$name.$r.err"
    echo "$name round $r: $(tail -c 300 "$OUT/$name.$r.out" | tr '\n' ' ' | cut -c1-200)"
  done
done
