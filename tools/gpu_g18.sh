# non-fused assembly writes the solver image (config 5, mode 2): stamps, bit A/B vs the round-4 start, BA + distributed GPU tests, bench
mkdir -p gpurun_out
true && \
timeout -k 10 300 python -u tools/ab_bits.py tools/abl/ts/libme_hip.so tools/abl/tsnoimg/libme_hip.so > gpurun_out/ab18.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_distributed.py tests/test_ba_mono_cov.py tests/test_pose_cov.py > gpurun_out/t18.log 2>&1
rc=$?; cat gpurun_out/ts18.log gpurun_out/ab18.log | grep -v amdgpu.ids; tail -3 gpurun_out/t18.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t18.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g18.json 2> gpurun_out/bench_g18.err
rc=$?; tail -2 gpurun_out/bench_g18.err; exit $rc
