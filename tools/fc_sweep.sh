set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for f in 8 6 4 10 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --mi-pairs 0 --pipeline-frames 0 --sharded-ba 0 --vo-matches 0 --front-cus $f > gpurun_out/fc_$f.log 2>&1 || exit 1
  echo "front_cus $f: $(grep -o '"value": [0-9.]*' gpurun_out/fc_$f.log)"
done
