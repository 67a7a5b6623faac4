# MI quad kernel, packed marginal words: parity tests, timing vs the byte-marginal build (two rounds), SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mi" --timeout 120 --timeout-method thread > gpurun_out/g27_t.log 2>&1; rc=$?; tail -3 gpurun_out/g27_t.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/g27_t.log; exit 1; }
for r in 1 2; do
  echo "pack:"; timeout -k 10 120 python tools/mi_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "nopack:"; timeout -k 10 120 python tools/mi_bench.py --check 0 --lib tools/abl/nopack/libme_hip.so 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/mi_pmc.sh > /dev/null
