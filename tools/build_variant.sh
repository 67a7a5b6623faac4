#!/bin/bash
# Build libme_hip.so with extra -D flags into tools/abl/<name>/ (A/B timing: bench.py --lib).
# Usage: tools/build_variant.sh NAME -DFOO=1 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../uasl_motion_estimation_amd/csrc"
out=../../tools/abl/$name
mkdir -p $out/obj
for f in api mi scale ba klt nms vo patch_ops; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "$@" -c $f.hip -o $out/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libme_hip.so $out/obj/*.o
rm -rf $out/obj
