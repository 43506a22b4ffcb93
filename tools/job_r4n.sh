set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
for L in d32 d96; do
  export DNN_HIP_LIB=diag/libdnn_hip_$L.so
  timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=1,2 --rounds 4 --iters 10 --kernels conv1 > $O/ab_$L.log 2>&1 || { tail -20 $O/ab_$L.log; exit 1; }
  echo "== $L"; grep "^{\"DNN" $O/ab_$L.log | cut -c1-900
done
