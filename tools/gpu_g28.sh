# MI quad kernel: walk loads in flight per lane (QUAD_U 4 default vs 2 / 6 / 8), two rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  for v in def u2 u6 u8; do
    if [ $v = def ]; then L=""; else L="--lib tools/abl/$v/libme_hip.so"; fi
    echo -n "$v: "; timeout -k 10 120 python tools/mi_bench.py --check 0 $L 2>&1 | grep pairs || exit 1
  done
done
