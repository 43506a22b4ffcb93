set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4zk; mkdir -p $O
timeout -k 10 300 python -u tools/lat_ab.py --env "DNN_HIP_KN=;4;43;45;435" --rounds 8 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep "graph_device" $O/lat.log | grep -v '^{"{' | cut -c1-700
