#!/bin/bash
# GPU check cycle used during development: parity tests, bench line, kernel trace
# (no event timing, for the frame timeline) and the PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --timing none --mi-pairs 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_trace.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && bash tools/pmc.sh
