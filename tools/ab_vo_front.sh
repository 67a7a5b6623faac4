#!/bin/bash
# A/B of the VO loop's front-end CU share (ME_VO_FRONT_CUS of every 16, whole XCDs): config-3 and config-5 loop lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for r in 1 2; do
  for f in 4 2 6; do
    k=$((k+1))
    ME_VO_FRONT_CUS=$f timeout -k 10 300 python bench.py --no-cpu-baseline --mi-pairs 0 --sharded-ba 0 --vo-matches 0 --steps 5 > gpurun_out/abf_$k.log 2>&1 || exit 1
    echo "[front $f] pipeline $(grep -o '"pipeline": {[^}]*}' gpurun_out/abf_$k.log | grep -o 'frames_per_s": [0-9.]*') c5 $(grep -o '"pipeline_config5": {[^}]*}' gpurun_out/abf_$k.log | grep -o 'frames_per_s": [0-9.]*')"
  done
done
