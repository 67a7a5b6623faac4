#!/bin/bash
# Headline bench (no CPU leg, no side lines) with the in-tree library vs variant builds, alternating.
# Usage (on the GPU box): tools/ab_lib.sh tools/abl/NAME/libme_hip.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for r in 1 2; do
  for l in default "$@"; do
    k=$((k+1))
    a=""; [ "$l" != default ] && a="--lib $l"
    timeout -k 10 200 python bench.py --no-cpu-baseline --mi-pairs 0 --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 $a > gpurun_out/abl_$k.log 2>&1 || exit 1
    echo "[$l] $(grep -o '"value": [0-9.]*' gpurun_out/abl_$k.log)"
  done
done
