# round-4 GPU step: VO loop with BA(t) chained behind BA(t-1) on the device (me_vo_ba_chain): pipeline GPU tests, bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/t10.log 2>&1
rc=$?; tail -8 gpurun_out/t10.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t10.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g10.json 2> gpurun_out/bench_g10.err
rc=$?; tail -3 gpurun_out/bench_g10.err; exit $rc
