# round-4 GPU step: cam_solve phases after the batched load, BA / pipeline / sharded GPU tests, a short bench line
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts2.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  tests/test_pipeline.py tests/test_distributed.py tests/test_ba_mono_cov.py > gpurun_out/t2.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
rc=$?
cat gpurun_out/solve_ts2.log; tail -15 gpurun_out/t2.log; tail -c 400 gpurun_out/bench_g2.json; tail -3 gpurun_out/bench_g2.err; exit $rc
