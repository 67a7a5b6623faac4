# assembly load batch (ME_SA_BATCH 8 / 16 / 32) on the image path: BA family times, two rounds
mkdir -p gpurun_out
for r in 1 2; do
  TAG=b16 timeout -k 10 200 python -u tools/ab_schur.py 2>/dev/null | grep -E "c3|c4" || exit 1
  TAG=b8 LIB=tools/abl/sab8/libme_hip.so timeout -k 10 200 python -u tools/ab_schur.py 2>/dev/null | grep -E "c3|c4" || exit 1
  TAG=b32 LIB=tools/abl/sab32/libme_hip.so timeout -k 10 200 python -u tools/ab_schur.py 2>/dev/null | grep -E "c3|c4" || exit 1
done
