set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3 or chain or tile or latency or net or batch or small" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/lat_ab.py --rounds 6 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | cut -c1-700
grep -A11 "plan:" $O/lat.log | head -12
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lt -o lt --output-format csv -- python3 $R/tools/lat_ab.py --rounds 1 --reps 100 > $O/lt.log 2>&1) || { tail -20 $O/lt.log; exit 1; }
python tools/trace_timeline.py $(find $O/lt -name "*kernel_trace.csv") --len 12 --reps 100
for L in d32 d96; do
  export DNN_HIP_LIB=diag/libdnn_hip_$L.so
  timeout -k 10 300 python tools/x3_ab.py --env DNN_HIP_X3_C16P=1,2 --rounds 4 --iters 10 --kernels conv1 > $O/ab_$L.log 2>&1 || { tail -20 $O/ab_$L.log; exit 1; }
  echo "== $L"; grep "^{\"DNN" $O/ab_$L.log | cut -c1-900
done
