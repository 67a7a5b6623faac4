#!/bin/bash
# HBM traffic per kernel launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (TCC slots), kernel-trace only, each pass under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 1 --no-cpu-baseline "$@" > "$OUT/$C.log" 2>&1 || exit 1
done
