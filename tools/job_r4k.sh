set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3 or chain or tile or avx or fuzz" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/lat_ab.py --env "DNN_AB_DUMMY=a;b" --rounds 6 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "^{\"DNN" $O/lat.log | grep graph | cut -c1-900
grep -A14 "plan:" $O/lat.log | head -16
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lt -o lt -- python tools/lat_ab.py --rounds 1 --reps 100 > $O/lt.log 2>&1 || { tail -20 $O/lt.log; exit 1; }
python tools/trace_timeline.py $(find $O/lt -name "*kernel_trace.csv") --len 12 --reps 100
