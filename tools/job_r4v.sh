set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4v; mkdir -p $O
timeout -k 10 300 python -u tools/lat_ab.py --rounds 8 --env "DNN_HIP_LAT_C16=;1" --env "DNN_AB_DUMMY=a;b" > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v "^{\"{" | cut -c1-330
