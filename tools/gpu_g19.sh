# fused mode-1 solve (config 4) on the assemblers' image: bit A/B, BA family times (config 4), BA GPU tests
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bits.py tools/abl/ts/libme_hip.so tools/abl/tsnoimg/libme_hip.so > gpurun_out/ab19.log 2>&1 && \
TAG=img timeout -k 10 200 python -u tools/ab_schur.py > gpurun_out/abs19.log 2>&1 && \
TAG=noimg LIB=tools/abl/tsnoimg/libme_hip.so timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs19.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_distributed.py tests/test_ba_mono_cov.py tests/test_pose_cov.py > gpurun_out/t19.log 2>&1
rc=$?; cat gpurun_out/ab19.log gpurun_out/abs19.log | grep -v amdgpu.ids; tail -3 gpurun_out/t19.log; exit $rc
