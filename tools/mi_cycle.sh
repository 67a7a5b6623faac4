#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mi_" --timeout 120 --timeout-method thread > gpurun_out/mi_t.log 2>&1; rc=$?; tail -3 gpurun_out/mi_t.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/mi_t.log; exit 1; }
timeout -k 10 120 python tools/mi_bench.py > gpurun_out/mi_quad.log 2>&1 && cat gpurun_out/mi_quad.log || exit 1
ME_MI_KERNEL=lane timeout -k 10 120 python tools/mi_bench.py --check 0 > gpurun_out/mi_lane.log 2>&1 && cat gpurun_out/mi_lane.log || exit 1
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_t.log 2>&1; rc=$?; tail -3 gpurun_out/pipe_t.log; exit $rc
