# DPP group reductions in pt_schur / pt_step: A/B timing (ab_schur), GPU tests, bench
mkdir -p gpurun_out
TAG=dpp timeout -k 10 200 python -u tools/ab_schur.py > gpurun_out/abs21.log 2>&1 && \
TAG=shfl LIB=tools/abl/dppoff/libme_hip.so timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs21.log 2>&1 && \
TAG=dpp timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs21.log 2>&1 && \
TAG=shfl LIB=tools/abl/dppoff/libme_hip.so timeout -k 10 200 python -u tools/ab_schur.py >> gpurun_out/abs21.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t21.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/abs21.log; tail -2 gpurun_out/t21.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t21.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g21.json 2> gpurun_out/bench_g21.err
rc=$?; tail -1 gpurun_out/bench_g21.err; exit $rc
