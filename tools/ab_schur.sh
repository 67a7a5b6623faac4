#!/bin/bash
# GPU tests, then tools/ab_schur.py over Schur variants (env / variant builds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
  tail -1 gpurun_out/t.log
fi
for r in 1 2; do
  TAG=sort timeout -k 10 200 python tools/ab_schur.py || exit 1
  TAG=nosort ME_SCHUR_SORT=0 timeout -k 10 200 python tools/ab_schur.py || exit 1
  for v in "$@"; do
    TAG=$v LIB=tools/abl/$v/libme_hip.so timeout -k 10 200 python tools/ab_schur.py || exit 1
  done
done
