#!/bin/bash
# Build libme_hip.so with extra -D flags into tools/abl/<name>/ (A/B timing: bench.py --lib).
# Same sources and link line as uasl_motion_estimation_amd/csrc/Makefile.
# Usage: tools/build_variant.sh NAME -DFOO=1 ...
set -e
name=$1; shift
cd "$(dirname "$0")/../uasl_motion_estimation_amd/csrc"
out=../../tools/abl/$name
mkdir -p $out/obj
SRC=$(sed -n 's/^SRC = //p' Makefile)
HOSTSRC=$(sed -n 's/^HOSTSRC = //p' Makefile)
for f in $SRC; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w "$@" -c $f -o $out/obj/${f%.hip}.o &
done
for f in $HOSTSRC; do
  g++ -std=c++17 -O3 -fPIC -w -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include "$@" -c $f -o $out/obj/${f%.cpp}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libme_hip.so $out/obj/*.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx
rm -rf $out/obj
