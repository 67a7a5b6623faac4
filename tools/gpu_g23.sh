# round-4 final evidence: all GPU tests, smoke, bench, profile cycle r04_c, 10k-keyframe run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t23.log 2>&1 || { tail -30 gpurun_out/t23.log; exit 1; }
tail -1 gpurun_out/t23.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke23.log 2>&1 || { tail -20 gpurun_out/smoke23.log; exit 1; }
tail -1 gpurun_out/smoke23.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_g23.json 2> gpurun_out/bench_g23.err || { tail -20 gpurun_out/bench_g23.err; exit 1; }
grep '^{' gpurun_out/bench_g23.json | cut -c1-200
bash tools/prof_cycle.sh r04_c > gpurun_out/prof_r04_c.log 2>&1 || { tail -30 gpurun_out/prof_r04_c.log; exit 1; }
grep -E "cam_solve|pt_schur|pt_step|linearize" gpurun_out/r04_c/kernel_stats.txt
timeout -k 10 1000 python -u tools/long_run.py --frames 10000 --out gpurun_out/r04_long_c5_10k_c.json > gpurun_out/r04_long_c.log 2>&1 || { tail -10 gpurun_out/r04_long_c.log; exit 1; }
tail -1 gpurun_out/r04_long_c.log | cut -c1-400
