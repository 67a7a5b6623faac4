# round-4 GPU step: cam_solve with the assemblers writing the LDS image (LDS-DMA copy): stamps, BA GPU tests, bench
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts5.log 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "ba_" \
  tests/test_gpu_parity.py tests/test_distributed.py > gpurun_out/t5.log 2>&1
rc=$?
cat gpurun_out/solve_ts5.log; tail -8 gpurun_out/t5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pipe_hostprof.py 3 40 > gpurun_out/hostprof5.log 2>&1; timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g5.json 2> gpurun_out/bench_g5.err
rc=$?; tail -3 gpurun_out/bench_g5.err; exit $rc
