# round-4 GPU step: register-resident panel (A/B stamps + bit A/B vs the LDS panel), BA GPU tests
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts7.log 2>&1 && \
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/tsold/libme_hip.so > gpurun_out/solve_ts7old.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bits.py tools/abl/ts/libme_hip.so tools/abl/tsold/libme_hip.so > gpurun_out/ab7.log 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "ba_" > gpurun_out/t7.log 2>&1
rc=$?
cat gpurun_out/solve_ts7.log gpurun_out/solve_ts7old.log gpurun_out/ab7.log; tail -4 gpurun_out/t7.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/t6.log 2>&1
rc=$?; tail -5 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g7.json 2> gpurun_out/bench_g7.err
rc=$?; tail -3 gpurun_out/bench_g7.err; exit $rc
