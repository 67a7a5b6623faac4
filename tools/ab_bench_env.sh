#!/bin/bash
# Headline bench (no CPU leg, no side lines) under several env settings, alternating: A/B timing.
# Usage (on the GPU box): tools/ab_bench_env.sh "VAR=val ..." "VAR=val ..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for e in "$@" "$@"; do
  k=$((k+1))
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --mi-pairs 0 --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 > gpurun_out/ab_$k.log 2>&1 || exit 1
  echo "[$e] $(grep -o '"value": [0-9.]*' gpurun_out/ab_$k.log) $(grep -o '"BA_SOLVE": {[^}]*}' gpurun_out/ab_$k.log)"
done
