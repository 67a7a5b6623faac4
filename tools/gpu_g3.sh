# round-4 GPU step: finer cam_solve load stamps, then a bench line (pipeline parity after the loop change)
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts3.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g3.json 2> gpurun_out/bench_g3.err
rc=$?
cat gpurun_out/solve_ts3.log; tail -3 gpurun_out/bench_g3.err; exit $rc
