set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fp16 or patch16" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python tools/x3_ab.py --precision fp16 --env DNN_HIP_P16V=1,2,3 --env DNN_AB_DUMMY=a,b --rounds 8 --iters 10 --kernels conv5,conv6,conv7,conv8 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep '^{"DNN' $O/ab.log | cut -c1-420
