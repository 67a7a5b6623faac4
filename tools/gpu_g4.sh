# round-4 GPU step: cam_solve load stamps, mono VO parity tests, a bench line (pipeline parity after the loop change)
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/solve_ts.py tools/abl/ts/libme_hip.so > gpurun_out/solve_ts3.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_mono_vo.py tests/test_cpp_adapter.py > gpurun_out/t4.log 2>&1
rc=$?
cat gpurun_out/solve_ts3.log; tail -15 gpurun_out/t4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g4.json 2> gpurun_out/bench_g4.err
rc=$?; tail -3 gpurun_out/bench_g4.err; exit $rc
