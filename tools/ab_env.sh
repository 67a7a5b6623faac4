#!/bin/bash
# rocprofv3 kernel stats of tools/ab_ba_fams.py for one config under several env settings.
# Usage (on the GPU box): tools/ab_env.sh CONFIG "VAR=val ..." "VAR=val ..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
cfg=$1; shift
k=0
for e in "$@"; do
  k=$((k+1)); d="$GRAFT_REPO_ROOT/gpurun_out/abe_$k"; rm -rf "$d"
  (cd /tmp && export TMPDIR=/tmp CONFIGS=$cfg $e && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 "$GRAFT_REPO_ROOT/tools/ab_ba_fams.py" > "$d.log" 2>&1) || exit 1
  echo "== $e"; grep "final" "$d.log" | cut -c1-160; python tools/kstats.py "$d/run_results.db" 6
done
