set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3_latency_kernel" > $O/pytest1.log 2>&1; rc=$?
tail -2 $O/pytest1.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest1.log | head -20; exit 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ktile or latency or x3_lat or tile or small or golden or conv3_shape" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/lat_ab.py --rounds 6  > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v "^{\"{" | cut -c1-700
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lt -o lt --output-format csv -- python3 $R/tools/lat_ab.py --rounds 1 --reps 100 > $O/lt.log 2>&1) || { tail -20 $O/lt.log; exit 1; }
python tools/trace_timeline.py $(find $O/lt -name "*kernel_trace.csv") --len 11 --reps 100
