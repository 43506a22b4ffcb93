set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4k2; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/lt -o lt --output-format csv -- python3 $R/tools/lat_ab.py --rounds 1 --reps 100 > $O/lt.log 2>&1) || { tail -20 $O/lt.log; exit 1; }
python tools/trace_timeline.py $(find $O/lt -name "*kernel_trace.csv") --len 12 --reps 100
