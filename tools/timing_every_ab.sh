set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "--timing-every 8" "--timing-every 32" "--timing none" "--timing-every 8" "--timing-every 32" "--timing none"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --mi-pairs 0 --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 $a > gpurun_out/te.log 2>&1 || exit 1
  echo "[$a] $(grep -o '"value": [0-9.]*' gpurun_out/te.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/te.log | head -1) $(grep -o '"timed_launches": [0-9]*' gpurun_out/te.log)"
done
