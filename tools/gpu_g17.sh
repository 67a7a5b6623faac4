# camera solve: is the diagonal block slowed by the worker waves? stamps with the trailing updates
# skipped (ME_SOLVE_SKIP=4, timing only) and with wave 0 at raised priority
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/ts17.log 2>&1 && \
ME_SOLVE_SKIP=4 timeout -k 10 200 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/ts17skip.log 2>&1 && \
timeout -k 10 200 python -u tools/solve_ts.py tools/abl/tsprio/libme_hip.so > gpurun_out/ts17prio.log 2>&1
rc=$?; grep "config 3" gpurun_out/ts17.log gpurun_out/ts17skip.log gpurun_out/ts17prio.log; exit $rc
