# VO loop front-end CU share A/B (ME_VO_FRONT_CUS of 16), two runs each, config 3 and 5
mkdir -p gpurun_out
for r in 1 2; do
  for f in 4 6 8; do
    for c in 3 5; do
      ME_VO_FRONT_CUS=$f timeout -k 10 200 python3 tools/pipe_run.py $c 40 2>/dev/null | grep -E "^config" | sed "s/^/front $f run $r: /" || exit 1
    done
  done
done
