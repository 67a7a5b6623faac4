#!/bin/bash
# A/B of an env setting on the headline bench (per-family BA times) and the
# config-3 / config-5 pipeline lines.  Usage: tools/ab_spec.sh VAR V1 V2 ...
# ("-" = VAR unset).  C5=frames enables the config-5 pipeline line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$1; shift
for v in "$@"; do
  if [ "$v" = "-" ]; then E="env -u $V"; else E="env $V=$v"; fi
  $E timeout -k 10 200 python bench.py --no-cpu-baseline --mi-pairs 0 --pipeline-frames ${C3:-40} --pipeline-c5-frames ${C5:-0} --sharded-ba 0 --vo-matches 0 > "gpurun_out/ab_$v.log" 2>&1 || { tail -20 "gpurun_out/ab_$v.log"; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")][0])
kb = {k: x["us_per_launch"] for k, x in (d.get("kernel_budget_per_frame") or {}).items()}
print(v, d["value"], kb, flush=True)
for key in ("pipeline", "pipeline_config5"):
    p = d.get(key) or {}
    if p: print(" ", key, p.get("frames_per_s"), p.get("host_ms_per_frame"), p.get("device_us_per_frame"), flush=True)
PY
done
