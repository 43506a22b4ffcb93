set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r4r; mkdir -p $O
timeout -k 10 300 python -u tools/lat_ab.py --rounds 6 --env "DNN_HIP_KT_NB=3;5" > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v "^{\"{" | cut -c1-700
export DNN_HIP_LIB=diag/libdnn_hip_d256.so
timeout -k 10 300 python -u tools/lat_ab.py --rounds 3 --env "DNN_HIP_KT_NB=3;5" > $O/lat256.log 2>&1 || { tail -20 $O/lat256.log; exit 1; }
grep -o '"DNN_HIP_KT_NB": "[0-9]"} {"graph_device_ms_median": [0-9.]*\|"ktile_stamps_us_last_round".*' $O/lat256.log | cut -c1-600
