#!/bin/bash
# Named GPU measurement steps, run in order; the first failing step ends the call.
#   tools/gpu_measure.sh STEP [STEP ...]
# steps: diag_ub (tools/abl/ubench_diag_g*), solve_ts:<variant> (tools/solve_ts.py on tools/abl/<variant>),
#        scale_ts:<variant>[:front_cus] (tools/scale_ts.py), klt (tools/klt_bench.py),
#        klt[:<variant>] (tools/klt_bench.py, bit-exact check), klt_sq (SQ counters of klt_kernel -> profiles/<tag>), mi (tools/mi_bench.py)
# Output: gpurun_out/measure_<step>.log (tail printed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${MEASURE_TAG:-r05}
for st in "$@"; do
  IFS=: read -r name a b <<< "$st"
  log="gpurun_out/measure_${name}${a:+_$a}${b:+_$b}.log"
  case "$name" in
    diag_ub) for x in tools/abl/ubench_diag_g*; do echo "$x"; timeout -k 5 60 "$x" || exit 1; done > "$log" 2>&1 ;;
    solve_ts) timeout -k 10 240 python3 tools/solve_ts.py "tools/abl/$a/libme_hip.so" > "$log" 2>&1 ;;
    scale_ts) timeout -k 10 240 python3 tools/scale_ts.py "tools/abl/$a/libme_hip.so" ${b:-0} > "$log" 2>&1 ;;
    klt) timeout -k 10 120 python3 tools/klt_bench.py ${a:+--lib tools/abl/$a/libme_hip.so} > "$log" 2>&1 ;;
    klt_sq) bash tools/sq_pmc.sh "${TAG}_klt_sq_counters" klt_kernel 2000 -- python3 "$GRAFT_REPO_ROOT/tools/klt_bench.py" --reps 5 --check 0 > "$log" 2>&1 ;;
    mi) timeout -k 10 120 python3 tools/mi_bench.py > "$log" 2>&1 ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  rc=$?
  echo "== $st (rc $rc)"; grep -v "amdgpu.ids" "$log" | tail -12
  [ $rc -eq 0 ] || exit $rc
done
