#!/bin/bash
# Diagnostic variants of libdnn_hip.so (wrong results, timing only): kernels_x3.hip rebuilt with
# -DX3DIAG=D for each D given, linked with the main build's other objects into
# dnn-inference-engine_amd/diag/libdnn_hip_dD.so (select with DNN_HIP_LIB=diag/libdnn_hip_dD.so).
set -e
cd "$(dirname "$0")/../dnn-inference-engine_amd/csrc"
make -j8 >/dev/null
mkdir -p ../diag build/diag
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -fno-slp-vectorize"
OBJS=$(ls build/*.o | grep -v kernels_x3.o | grep -v abi_avx.o)
for D in "$@"; do
  ( /opt/rocm/bin/hipcc $FL -DX3DIAG=$D -c kernels_x3.hip -o build/diag/kernels_x3_d$D.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../diag/libdnn_hip_d$D.so $OBJS build/diag/kernels_x3_d$D.o ) &
done
wait
ls -la ../diag
