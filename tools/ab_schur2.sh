#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  TAG=new timeout -k 10 200 python tools/ab_schur.py || exit 1
  TAG=old LIB=tools/abl/old/libme_hip.so timeout -k 10 200 python tools/ab_schur.py || exit 1
done
timeout -k 10 300 python tools/pipe_hostprof.py 3 40 > gpurun_out/hostprof.txt 2>&1 || exit 1
head -5 gpurun_out/hostprof.txt
