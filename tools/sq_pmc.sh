#!/bin/bash
# SQ counter passes (one --pmc pass each, kernel-trace only, each under its own time limit) over a
# driver command, summarised for one kernel by tools/sq_summary.py into profiles/<TAG>.txt/.json.
#   tools/sq_pmc.sh TAG KERNEL_REGEX UNITS -- python3 tools/klt_bench.py --reps 5 --check 0
# UNITS: the work units per launch the per-unit figures are quoted for (e.g. 2000 features).
set -o pipefail
TAG=$1; RX=$2; UNITS=$3; shift 3; [ "$1" = "--" ] && shift
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES"
P3="SQ_WAIT_INST_ANY SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE"
for p in P1 P2 P3; do
  timeout -s KILL 90 rocprofv3 --pmc ${!p} --output-format csv -d "$OUT/$p" -o run -- "$@" > "$OUT/$p.log" 2>&1 \
    || { tail -5 "$OUT/$p.log"; exit 1; }
done
cd "$GRAFT_REPO_ROOT" && python3 tools/sq_summary.py "$TAG" "$RX" "$UNITS" "$OUT"
