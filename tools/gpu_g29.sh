# MI quad kernel: walk state as LDS byte offsets vs the previous commit (two rounds), parity tests, SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_pipeline.py -x -q -k "mi or epipolar" --timeout 120 --timeout-method thread > gpurun_out/g29_t.log 2>&1; rc=$?; tail -3 gpurun_out/g29_t.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/g29_t.log; exit 1; }
for r in 1 2; do
  echo -n "new:  "; timeout -k 10 120 python tools/mi_bench.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' '; echo
  echo -n "prev: "; timeout -k 10 120 python tools/mi_bench.py --check 0 --lib tools/abl/prev/libme_hip.so 2>&1 | grep pairs || exit 1
done
bash tools/mi_pmc.sh > /dev/null
