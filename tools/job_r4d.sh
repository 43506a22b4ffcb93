set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chain or c16 or golden or x3_conv or tile_placement" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=0,1,2 --rounds 4 --kernels conv0,conv1,conv2 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
head -3 $O/ab.log | cut -c1-400
