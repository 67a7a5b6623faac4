#!/bin/bash
# GPU-box steps (run through gpurun).  Every GPU step runs under its own time
# limit, steps are chained with &&, and the first failure ends the call.
#   tools/gpu.sh final                      GPU tests, smoke, default bench line (gpurun_out/final_*)
#   tools/gpu.sh prof TAG [BENCH ARGS]      rocprofv3 --kernel-trace --stats of the headline bench frame
#                                           (no event timing) + FETCH_SIZE / WRITE_SIZE --pmc passes
#                                           (gpurun_out/TAG/; summarise with tools/summarise.py kstats / pmc)
#   tools/gpu.sh benchprof TAG              rocprofv3 --kernel-trace --stats of the full default bench command
#   tools/gpu.sh sq TAG KERNEL_RX UNITS UNIT -- CMD...
#                                           SQ counter passes (one --pmc pass each) over CMD, summarised
#                                           into profiles/TAG.txt / .json (tools/summarise.py sq)
#   tools/gpu.sh ab [-k PYTEST_EXPR] [-r ROUNDS] [-t TAG] -- CMD...
#                                           GPU tests (-k selection), then ROUNDS interleaved runs of CMD with
#                                           this tree's library and with every tools/abl/<v>/libme_hip.so
#                                           (ME_LIB), log in gpurun_out/ab_TAG.log
#   tools/gpu.sh coop                       plain vs cooperative-launch build (tools/abl/coop, built with
#                                           tools/build_variant.sh coop -DME_COOP_LAUNCH=1): wall clocks and
#                                           kernel stats of tools/drivers.py coop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cmd=$1; shift
case "$cmd" in
  final)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 && tail -3 gpurun_out/final_tests.log &&
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 && tail -1 gpurun_out/final_smoke.log &&
    timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err && tail -1 gpurun_out/final_bench.json | cut -c1-400
    ;;
  prof)
    TAG=$1; shift
    OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
    ARGS="--no-cpu-baseline --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 --streams 1 $*"
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$R/bench.py" --timing none $ARGS > "$OUT/stats.log" 2>&1 &&
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc/FETCH_SIZE" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 $ARGS > "$OUT/pmc_FETCH_SIZE.log" 2>&1 &&
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc/WRITE_SIZE" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 $ARGS > "$OUT/pmc_WRITE_SIZE.log" 2>&1 &&
    cd "$R" && python3 tools/summarise.py kstats "$(ls $OUT/stats/run_kernel_stats.csv $OUT/stats/*/run_kernel_stats.csv 2>/dev/null | head -1)" 25
    ;;
  benchprof)
    TAG=$1
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/benchprof" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/${TAG}_benchprof.log" 2>&1 &&
    grep '^{' "$R/gpurun_out/${TAG}_benchprof.log" | cut -c1-300
    ;;
  sq)
    TAG=$1; RX=$2; UNITS=$3; UNIT=$4; shift 4; [ "$1" = "--" ] && shift
    OUT="$R/gpurun_out/sq_$TAG"; mkdir -p "$OUT"
    P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
    P2="SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES"
    P3="SQ_WAIT_INST_ANY SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE"
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/P1" -o run -- "$@" > "$OUT/P1.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/P2" -o run -- "$@" > "$OUT/P2.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc $P3 --output-format csv -d "$OUT/P3" -o run -- "$@" > "$OUT/P3.log" 2>&1 &&
    cd "$R" && python3 tools/summarise.py sq "$TAG" "$RX" "$UNITS" "$OUT" "$UNIT"
    ;;
  ab)
    K=""; ROUNDS=2; TAG=ab
    while [ $# -gt 0 ]; do
      case "$1" in
        -k) K="$2"; shift 2 ;;
        -r) ROUNDS="$2"; shift 2 ;;
        -t) TAG="$2"; shift 2 ;;
        --) shift; break ;;
        *) break ;;
      esac
    done
    SEL=(-m gpu); [ -n "$K" ] && SEL=(-m gpu -k "$K")
    LOG=gpurun_out/ab_$TAG.log; : > "$LOG"
    timeout -k 10 600 python -u -m pytest tests "${SEL[@]}" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/ab_${TAG}_tests.log; exit 1; }
    tail -1 gpurun_out/ab_${TAG}_tests.log
    [ $# -eq 0 ] && exit 0
    for r in $(seq 1 "$ROUNDS"); do
      echo "new:" >> "$LOG"
      timeout -k 10 300 "$@" >> "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
      for d in tools/abl/*/; do
        [ -f "$d/libme_hip.so" ] || continue
        echo "$(basename "$d"):" >> "$LOG"
        ME_LIB="$d/libme_hip.so" timeout -k 10 300 "$@" >> "$LOG" 2>&1 || { tail -20 "$LOG"; exit 1; }
      done
    done
    grep -vE 'amdgpu.ids' "$LOG" | cut -c1-400
    ;;
  coop)
    timeout -k 10 240 python -u tools/drivers.py coop > gpurun_out/coop_normal.json &&
    timeout -k 10 240 python -u tools/drivers.py --lib tools/abl/coop/libme_hip.so coop > gpurun_out/coop_coop.json &&
    cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/coop_normal_stats" -o run -- python3 "$R/tools/drivers.py" coop --reps 10 > "$R/gpurun_out/coop_normal_prof.log" 2>&1 &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/coop_coop_stats" -o run -- python3 "$R/tools/drivers.py" --lib "$R/tools/abl/coop/libme_hip.so" coop --reps 10 > "$R/gpurun_out/coop_coop_prof.log" 2>&1
    cat "$R/gpurun_out/coop_normal.json" "$R/gpurun_out/coop_coop.json"
    ;;
  *)
    sed -n '2,24p' "$0"; exit 2 ;;
esac
