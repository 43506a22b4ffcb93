set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 60 tools/launch_probe || exit 1
for L in main d32 d96 d160 d224; do
  if [ $L = main ]; then unset DNN_HIP_LIB; else export DNN_HIP_LIB=diag/libdnn_hip_$L.so; fi
  timeout -k 10 200 python tools/x3_ab.py --env DNN_AB_DUMMY=a --rounds 4 --iters 10 --preheat 2 --kernels conv0,conv1,conv2,conv3 > $O/ab_$L.log 2>&1 || { tail -20 $O/ab_$L.log; exit 1; }
  echo "== $L"; grep "^{\"DNN" $O/ab_$L.log | cut -c1-900
done
