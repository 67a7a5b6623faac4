# round-end sanity: full GPU suite, smoke, default bench on the committed tree
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 && tail -3 gpurun_out/final_tests.log &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 && tail -1 gpurun_out/final_smoke.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err && cat gpurun_out/final_bench.json
