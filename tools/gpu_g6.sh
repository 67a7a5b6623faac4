# round-4 GPU step: VO loop with the asynchronous scale LM and BA enqueue: pipeline GPU tests + bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/t6.log 2>&1
rc=$?; tail -8 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --cpu-runs 2 > gpurun_out/bench_g6.json 2> gpurun_out/bench_g6.err
rc=$?; tail -3 gpurun_out/bench_g6.err; exit $rc
