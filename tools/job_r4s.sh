set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4s; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ktile or latency or x3_lat or tile or small" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/lat_ab.py --rounds 6 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v "^{\"{" | cut -c1-700
export DNN_HIP_LIB=diag/libdnn_hip_d256.so
timeout -k 10 300 python -u tools/lat_ab.py --rounds 3 > $O/lat256.log 2>&1 || { tail -20 $O/lat256.log; exit 1; }
grep -o '"ktile_stamps_us_last_round".*' $O/lat256.log | head -1 | cut -c1-400
