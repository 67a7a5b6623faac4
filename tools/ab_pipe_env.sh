#!/bin/bash
# VO-loop bench lines (configs 3 and 5) under env variants, alternating.
# Usage: tools/ab_pipe_env.sh "ENV=1 ..." ["ENV2=..."]   ("-" = no env)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
k=0
for r in 1 2; do
  for e in - "$@"; do
    k=$((k+1))
    [ "$e" = - ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --mi-pairs 0 --sharded-ba 0 --vo-matches 0 --steps 5 --warmup 2 > gpurun_out/abp_$k.log 2>&1 || { tail -5 gpurun_out/abp_$k.log; exit 1; }
    python - "$e" gpurun_out/abp_$k.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
p3, p5 = d.get("pipeline") or {}, d.get("pipeline_config5") or {}
print(f"[{sys.argv[1] or 'default'}] c3 {p3.get('frames_per_s')} f/s host {p3.get('host_ms_per_frame')} BA_SCHUR {p3.get('device_us_per_frame', {}).get('BA_SCHUR')} | c5 {p5.get('frames_per_s')} f/s BA_SCHUR {p5.get('device_us_per_frame', {}).get('BA_SCHUR')} BA_SOLVE {p5.get('device_us_per_frame', {}).get('BA_SOLVE')}")
PY
  done
done
