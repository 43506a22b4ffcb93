set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
DNN_HIP_LIB=diag/libdnn_hip_d16.so timeout -k 10 300 python tools/x3_ab.py --rounds 3 --preheat 4 > $O/ab_d16.log 2>&1 || { tail -20 $O/ab_d16.log; exit 1; }
tail -1 $O/ab_d16.log
