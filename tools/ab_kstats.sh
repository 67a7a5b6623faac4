#!/bin/bash
# rocprofv3 kernel stats of tools/ab_ba_fams.py for one config, default library vs variants.
# Usage (on the GPU box): tools/ab_kstats.sh CONFIG VARIANT...   (tools/abl/<VARIANT>/libme_hip.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
cfg=$1; shift
for v in default "$@"; do
  lib=""; [ "$v" != default ] && lib="$GRAFT_REPO_ROOT/tools/abl/$v/libme_hip.so"
  d="$GRAFT_REPO_ROOT/gpurun_out/abk_$v"
  rm -rf "$d"
  (cd /tmp && TMPDIR=/tmp LIB=$lib CONFIGS=$cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 "$GRAFT_REPO_ROOT/tools/ab_ba_fams.py" > "$d.log" 2>&1) || exit 1
  echo "== $v"; python tools/kstats.py "$d/run_results.db" 8
done
