#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   kernel trace + stats of the serialised n=1024 ceremony, then separate PMC passes
#   (SQ issue/wait counters; FETCH_SIZE; WRITE_SIZE; VALU thread-cycles vs instructions) -- never
#   combined with runtime/sys traces.
# usage: tools/profile.sh <tag> [extra bench args]
set -e -o pipefail
TAG=${1:-r01}
shift || true
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$REPO/bench.py --no-cpu --no-interp --streams 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B --steps 2 --warmup 1 > "$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $B --steps 1 --warmup 0 > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $B --steps 1 --warmup 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $B --steps 1 --warmup 0 > "$OUT/pmc_write.log" 2>&1
# the roofline's unit, measured: thread-cycles of VALU work (half-rate instructions take twice the
# cycles of full-rate ones) against instructions issued (tools/pmc_summary.py: slots per instruction)
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_valu" -o run -- python3 $B --steps 1 --warmup 0 > "$OUT/pmc_valu.log" 2>&1
echo done
