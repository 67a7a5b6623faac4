# VO loop with reserved BA buffers: timing probe, pipeline GPU tests, bench
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/pipe_run.py 3 40 > gpurun_out/prun13.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prun13.log | head -24; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/t13.log 2>&1
rc=$?; tail -8 gpurun_out/t13.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t13.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g13.json 2> gpurun_out/bench_g13.err
rc=$?; tail -3 gpurun_out/bench_g13.err; exit $rc
