# round-4 GPU step: cam_solve wall-clock phases (timing variant), the sharded tests, the native-4K
# front-end tests, the epipolar border test, then one short bench line (CPU legs pinned)
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py \
  "tests/test_gpu_configs.py::test_scale_config4_8000_tracks_native_4k" "tests/test_gpu_configs.py::test_klt_config4_8000_features_native_4k" \
  tests/test_pipeline.py > gpurun_out/dist.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g1.json 2> gpurun_out/bench_g1.err
rc=$?
cat gpurun_out/solve_ts.log; tail -30 gpurun_out/dist.log; tail -c 600 gpurun_out/bench_g1.json; tail -5 gpurun_out/bench_g1.err; exit $rc
