#!/bin/bash
# A/B of the front-end / BA CU split (ME_CU_SPLIT): composite frame and the config-3 VO loop line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for r in 1 2; do
  for e in "ME_CU_SPLIT=interleaved" "ME_CU_SPLIT=xcd"; do
    k=$((k+1))
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --mi-pairs 0 --sharded-ba 0 --vo-matches 0 > gpurun_out/abs_$k.log 2>&1 || exit 1
    echo "[$e] $(grep -o '"value": [0-9.]*' gpurun_out/abs_$k.log) pipeline $(grep -o '"pipeline": {[^}]*}' gpurun_out/abs_$k.log | grep -o 'frames_per_s": [0-9.]*') c5 $(grep -o '"pipeline_config5": {[^}]*}' gpurun_out/abs_$k.log | grep -o 'frames_per_s": [0-9.]*')"
  done
done
