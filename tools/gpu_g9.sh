# round-4 GPU step: E = L^-T backward (stamps A/B, bit A/B), speculative linearisation and
# 32-landmark Schur sub-chunks (tools/ab_schur.py A/B), BA GPU tests
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_ba_mono_cov.py tests/test_pose_cov.py tests/test_distributed.py > gpurun_out/t9.log 2>&1
rc=$?; tail -5 gpurun_out/t9.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t9.log | head -30; exit $rc; }
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts9.log 2>&1 && \
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/tsnoinv/libme_hip.so > gpurun_out/solve_ts9noinv.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bits.py tools/abl/ts/libme_hip.so tools/abl/tsold/libme_hip.so > gpurun_out/ab9.log 2>&1 && \
TAG=spec timeout -k 10 200 python -u tools/ab_schur.py > gpurun_out/abs9.log 2>&1 && \
TAG=nospec ME_BA_SPEC_LIN=0 timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs9.log 2>&1 && \
TAG=pts32 ME_SCHUR_PTS=32 timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs9.log 2>&1 && \
TAG=spec timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs9.log 2>&1
rc=$?
grep "config 3" gpurun_out/solve_ts9.log gpurun_out/solve_ts9noinv.log; cat gpurun_out/ab9.log gpurun_out/abs9.log | grep -v amdgpu.ids
exit $rc
