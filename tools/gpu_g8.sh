# round-4 GPU step: register backward solve + block 0 beside the LDS copy (stamps A/B, bit A/B), BA GPU tests
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts8.log 2>&1 && \
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/tsne/libme_hip.so > gpurun_out/solve_ts8ne.log 2>&1 && \
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/tsold/libme_hip.so > gpurun_out/solve_ts8old.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bits.py tools/abl/ts/libme_hip.so tools/abl/tsold/libme_hip.so > gpurun_out/ab8.log 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "ba_" > gpurun_out/t8.log 2>&1
rc=$?
cat gpurun_out/solve_ts8.log gpurun_out/solve_ts8ne.log gpurun_out/solve_ts8old.log gpurun_out/ab8.log; tail -4 gpurun_out/t8.log
exit $rc
