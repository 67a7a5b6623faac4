#!/bin/bash
# GPU check cycle used during development: parity tests, bench line, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
timeout -k 10 120 python tools_solve_stamps.py > gpurun_out/stamps.log 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.log" 2>&1
