#!/bin/bash
# One parameterised GPU A/B cycle (replaces the one-off gpu_g1..g29 lease scripts):
#   tools/gpu_ab.sh [-k PYTEST_EXPR] [-r ROUNDS] [-t TAG] -- CMD...
# 1. the GPU parity tests selected by -k (all of -m gpu when empty) on the tree's build;
# 2. ROUNDS interleaved runs of CMD against this tree's libme_hip.so ("new") and against
#    every prebuilt variant tools/abl/<v>/libme_hip.so (tools/build_variant.sh), passed to CMD
#    through ME_LIB (honoured by _lib.load_library); each run under its own time limit.
# Output under gpurun_out/ab_<TAG>.log.  Stops at the first failing step.
set -o pipefail
K=""; R=2; TAG=ab
while [ $# -gt 0 ]; do
  case "$1" in
    -k) K="$2"; shift 2 ;;
    -r) R="$2"; shift 2 ;;
    -t) TAG="$2"; shift 2 ;;
    --) shift; break ;;
    *) break ;;
  esac
done
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LOG=gpurun_out/ab_$TAG.log
SEL=(-m gpu); [ -n "$K" ] && SEL=(-m gpu -k "$K")
timeout -k 10 600 python -u -m pytest tests "${SEL[@]}" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_${TAG}_tests.log 2>&1 \
  || { tail -30 gpurun_out/ab_${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/ab_${TAG}_tests.log
[ $# -eq 0 ] && exit 0
: > "$LOG"
for r in $(seq 1 "$R"); do
  echo "new:" | tee -a "$LOG"
  timeout -k 10 300 "$@" >> "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
  for d in tools/abl/*/; do
    [ -f "$d/libme_hip.so" ] || continue
    v=$(basename "$d"); echo "$v:" | tee -a "$LOG"
    ME_LIB="$d/libme_hip.so" timeout -k 10 300 "$@" >> "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
  done
done
grep -E '^(new|[A-Za-z0-9_]+):|^\{' "$LOG" | cut -c1-400
