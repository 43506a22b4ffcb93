#!/bin/bash
# Experimental variants of libdnn_hip.so: kernels_x3.hip rebuilt with extra defines, linked with the
# main build's other objects into dnn-inference-engine_amd/diag/libdnn_hip_NAME.so (select with
# DNN_HIP_LIB=diag/libdnn_hip_NAME.so).  Arguments: D (a number: -DX3DIAG=D, diagnostic builds
# with wrong results, NAME = dD) or NAME:FLAGS (e.g. c0d2:-DC0DIAG=2); FILE=conv_small.hip for the
# conv0 diagnostics (default kernels_x3.hip).
set -e
cd "$(dirname "$0")/../dnn-inference-engine_amd/csrc"
make -j8 >/dev/null
mkdir -p ../diag build/diag
F=${FILE:-kernels_x3.hip}
B=${F%.hip}
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -fno-slp-vectorize"
[ "$F" = kernels_x3.hip ] || FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden"
OBJS=$(ls build/*.o | grep -v "$B.o" | grep -v abi_avx.o)
for A in "$@"; do
  case $A in
    *:*) N=${A%%:*}; DF=${A#*:} ;;
    *) N=d$A; DF=-DX3DIAG=$A ;;
  esac
  ( /opt/rocm/bin/hipcc $FL $DF -c $F -o build/diag/${B}_$N.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../diag/libdnn_hip_$N.so $OBJS build/diag/${B}_$N.o ) &
done
wait
ls -la ../diag
