#!/bin/bash
# Profiling cycle of the headline bench (round-tagged): rocprofv3 kernel-trace
# stats (no event timing), then the PMC traffic passes (FETCH_SIZE, WRITE_SIZE
# in separate runs, kernel-trace only).  Usage: tools/prof_cycle.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --timing none $ARGS > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
python3 "$GRAFT_REPO_ROOT/tools/kstats.py" "$(ls $OUT/stats/run_kernel_stats.csv $OUT/stats/*/run_kernel_stats.csv 2>/dev/null | head -1)" 40 > "$OUT/kernel_stats.txt" || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 1 $ARGS > "$OUT/pmc_$C.log" 2>&1 || exit 1
done
cd "$GRAFT_REPO_ROOT"
ls -R "$OUT" | head -30
cat "$OUT/kernel_stats.txt"
