set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3_latency or latency" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/lat_ab.py --rounds 6 > $O/lat0.log 2>&1 || { tail -20 $O/lat0.log; exit 1; }
grep "graph_device" $O/lat0.log | grep -v "^{\"{" | cut -c1-600
export DNN_HIP_LIB=diag/libdnn_hip_d512.so
timeout -k 10 300 python -u tools/lat_ab.py --rounds 3 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep -o '"lat_stamps_us_last_round".*' $O/lat.log | head -1 | cut -c1-400
