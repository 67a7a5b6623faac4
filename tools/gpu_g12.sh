# VO loop: BA enqueue vs completion times (unprofiled), chained and unchained
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/pipe_run.py 3 40 > gpurun_out/prun.log 2>&1 && \
ME_VO_CHAIN=0 timeout -k 10 200 python3 tools/pipe_run.py 3 40 > gpurun_out/prun0.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prun.log | head -20; grep -v amdgpu.ids gpurun_out/prun0.log | head -8; exit $rc
