set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
DNN_HIP_LIB=diag/libdnn_hip_d16.so timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_MG=1,4,2 > $O/ab_d16.log 2>&1 || { tail -20 $O/ab_d16.log; exit 1; }
tail -4 $O/ab_d16.log | head -3
timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_MG=1,4,2 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -4 $O/ab.log | head -3
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
