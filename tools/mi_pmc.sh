#!/bin/bash
# MI batch kernel: timing + self-check, then SQ counter passes (one --pmc pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mipmc
timeout -k 10 120 python3 tools/mi_bench.py "$@" > gpurun_out/mipmc/bench.log 2>&1 || { cat gpurun_out/mipmc/bench.log; exit 1; }
cat gpurun_out/mipmc/bench.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/mipmc/p1" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/mi_bench.py" --reps 2 --check 0 > "$GRAFT_REPO_ROOT/gpurun_out/mipmc/p1.log" 2>&1 || exit 1
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/mipmc/p2" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/mi_bench.py" --reps 2 --check 0 > "$GRAFT_REPO_ROOT/gpurun_out/mipmc/p2.log" 2>&1 || exit 1
