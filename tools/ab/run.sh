#!/bin/bash
# One GPU call from a recipe file (run on the GPU box from the repo root):
#   bash tools/ab/run.sh <recipe> [tag]
# A recipe is a text file of steps, one per line:   <name> <timeout_s> <command ...>
# ('#' starts a comment line; blank lines are skipped; $O in a command is the step output directory
# gpurun_out/<tag>, $R the repo root).  Each step runs under its own `timeout -k 10 <timeout_s>`
# with stdout+stderr in $O/<name>.log; its last 3 lines are echoed.  The call stops at the first
# failing step (a GPU fault, abort or time limit ends it there), so nothing runs after trouble.
# Recipes live in tools/ab/recipes/; tools/ab/ab.sh (interleaved A/B rounds) and tools/ab/build.sh
# (variant libraries under ab_build/) are commands a recipe step can call.
set -o pipefail
RECIPE=$1
TAG=${2:-$(basename "$RECIPE" .txt)}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export R O
while IFS= read -r line || [[ -n $line ]]; do
  [[ -z ${line// } || $line == \#* ]] && continue
  read -r name tmo cmd <<< "$line"
  echo "== $name (limit ${tmo}s)"
  start=$(date +%s)
  if ! timeout -k 10 "$tmo" bash -o pipefail -c "$cmd" > "$O/$name.log" 2>&1; then
    rc=$?
    echo "STEP $name FAILED (exit $rc after $(( $(date +%s) - start ))s)"
    tail -30 "$O/$name.log"
    exit 1
  fi
  echo "   ok in $(( $(date +%s) - start ))s: $(tail -3 "$O/$name.log" | cut -c1-240 | tr '\n' ' ')"
done < "$RECIPE"
echo ALL DONE
