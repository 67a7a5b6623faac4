# round-4 profile cycle: headline-frame rocprofv3 stats + PMC traffic passes (tools/prof_cycle.sh),
# kernel stats of the whole bench command, MI SQ counters, camera-solve stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/prof_cycle.sh r04_a > gpurun_out/prof_r04_a.log 2>&1 || { tail -30 gpurun_out/prof_r04_a.log; exit 1; }
tail -45 gpurun_out/prof_r04_a.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04_a/bstats" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r04_a/bench_prof.log" 2>&1) || { tail -20 gpurun_out/r04_a/bench_prof.log; exit 1; }
python3 tools/kstats.py "$(ls gpurun_out/r04_a/bstats/run_kernel_stats.csv gpurun_out/r04_a/bstats/*/run_kernel_stats.csv 2>/dev/null | head -1)" 40 > gpurun_out/r04_a/bench_kernel_stats.txt || true
grep '^{' gpurun_out/r04_a/bench_prof.log | cut -c1-200
bash tools/mi_pmc.sh > gpurun_out/r04_a/mi_pmc.log 2>&1 || { tail -20 gpurun_out/r04_a/mi_pmc.log; exit 1; }
tail -5 gpurun_out/r04_a/mi_pmc.log
