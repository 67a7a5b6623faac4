#!/bin/bash
# Round profile set: GPU tests, full bench line (CPU baseline included), rocprofv3
# stats of the bench command, headline kernel stats + PMC traffic (prof_cycle.sh),
# MI batch kernel SQ counters (mi_pmc.sh).  Usage: tools/prof_round.sh TAG
set -o pipefail
TAG=$1
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash tools/mi_pmc.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
rm -rf "$GRAFT_REPO_ROOT/gpurun_out/prof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && bash tools/prof_cycle.sh "$TAG"
