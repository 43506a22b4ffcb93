# batch-1 latency plan: GPU tests of the split combine, a sweep of the chooser's switches,
# then a rocprof kernel trace of the default latency plan
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "latency or splitk or yolo_batch1" > gpurun_out/pytest_lat.log 2>&1 || { tail -40 gpurun_out/pytest_lat.log; exit 1; }
tail -2 gpurun_out/pytest_lat.log
for cfg in "7 6" "1 6" "3 6" "5 6" "7 4" "7 3" "7 8"; do
  set -- $cfg
  DNN_HIP_LAT_CAND=$1 DNN_HIP_LAT_MINSTEPS=$2 timeout -k 10 120 python tools/lat_probe.py > gpurun_out/lat_$1_$2.log 2>&1 || { tail -20 gpurun_out/lat_$1_$2.log; exit 1; }
  echo "cand=$1 minsteps=$2"; tail -1 gpurun_out/lat_$1_$2.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['graph_ms'],d['graph_device_ms'],d['kernel_ms'])"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lat_trace -o trace --output-format csv -- python3 $R/tools/lat_probe.py > $R/gpurun_out/lat_trace.log 2>&1 || exit 1
echo LATOK
