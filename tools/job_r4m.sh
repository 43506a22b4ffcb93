set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3 or chain or tile or avx or fuzz or net" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=1,2 --env DNN_AB_DUMMY=a,b --rounds 6 --iters 10 --kernels conv0,conv1,conv2 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep "^{\"DNN" $O/ab.log | cut -c1-400
export DNN_HIP_LIB=diag/libdnn_hip_d32.so
timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=1,2 --rounds 4 --iters 10 --kernels conv1 > $O/ab32.log 2>&1 || { tail -20 $O/ab32.log; exit 1; }
grep "^{\"DNN" $O/ab32.log | cut -c1-900
