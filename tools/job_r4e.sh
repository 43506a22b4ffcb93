set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=0,2 --env DNN_AB_DUMMY=a,b --rounds 8 --iters 10 --kernels conv0,conv1,conv2,conv7 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep '^{"DNN' $O/ab.log | cut -c1-420
