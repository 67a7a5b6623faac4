#!/bin/bash
# Build timing-experiment variants of libme_hip.so into tools/exp/: MI_EXP=1..3, or mXY = MI_MREG=X MI_UCLR=Y.
set -e
cd "$(dirname "$0")/../uasl_motion_estimation_amd/csrc"
mkdir -p ../../tools/exp/obj
for E in ${VARIANTS:-1 2 3}; do
  case $E in
    m*) F="-DMI_MREG=${E:1:1} -DMI_UCLR=${E:2:1}" ;;
    p*) F="-DMI_PERM=${E:1}" ;;
    *) F="-DMI_EXP=$E" ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $F -c mi.hip -o ../../tools/exp/obj/mi$E.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/exp/libme_hip_exp$E.so build/api.o ../../tools/exp/obj/mi$E.o build/scale.o build/ba.o build/klt.o build/nms.o build/vo.o
done
