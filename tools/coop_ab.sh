#!/bin/bash
# Normal vs cooperative launch of scale_lm_kernel / cam_solve_kernel<2>.
# Needs tools/abl/coop/libme_hip.so (tools/build_variant.sh coop -DME_COOP_LAUNCH=1).
# Output: gpurun_out/coop_{normal,coop}.json (wall clocks) and gpurun_out/coop_{normal,coop}_stats/
# (rocprofv3 --kernel-trace --stats).  Every GPU step under its own time limit, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/coop_ab.py 20 > gpurun_out/coop_normal.json &&
ME_LIB=tools/abl/coop/libme_hip.so timeout -k 10 240 python -u tools/coop_ab.py 20 > gpurun_out/coop_coop.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/coop_normal_stats -o run -- python3 tools/coop_ab.py 10 > gpurun_out/coop_normal_prof.log 2>&1 &&
ME_LIB=tools/abl/coop/libme_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/coop_coop_stats -o run -- python3 tools/coop_ab.py 10 > gpurun_out/coop_coop_prof.log 2>&1 &&
cat gpurun_out/coop_normal.json gpurun_out/coop_coop.json
