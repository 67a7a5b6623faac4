#!/bin/bash
# Quick GPU cycle: GPU tests, bench line, no-event kernel trace of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline --mi-pairs 0 "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
rm -rf "$GRAFT_REPO_ROOT/gpurun_out/trace"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --timing none --mi-pairs 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_trace.log" 2>&1 || exit 1
