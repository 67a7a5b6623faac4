# round-4: linearize restored, staged read-back opt-in; GPU tests (BA, pipeline, mono, distributed), bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t14.log 2>&1
rc=$?; tail -3 gpurun_out/t14.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t14.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g14.json 2> gpurun_out/bench_g14.err
rc=$?; tail -2 gpurun_out/bench_g14.err; exit $rc
