set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3 or chain or tile or latency or net or small or ktile" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 400 python -u tools/lat_ab.py --rounds 6 --env "DNN_HIP_SPLIT=;1152:9;1152:12;2304:12;2304:18;2304:24;1152:12,2304:18,1024:8" > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v "^{\"{" | cut -c1-600
