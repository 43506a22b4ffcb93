# conv6/conv7 at batch 1: tile config x split sweep (DNN_HIP_CFG + DNN_HIP_SPLIT, batch-rule candidate only)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
export DNN_HIP_LAT_CAND=1 ITERS=100
for cs in "8 8" "8 16" "7 8" "7 12" "7 16" "7 24" "4 16" "4 32" "3 32" "14 16" "14 32" "14 24"; do
  set -- $cs
  DNN_HIP_CFG="9216:$1,4608:$1" DNN_HIP_SPLIT="9216:$2,4608:$2" timeout -k 10 60 python tools/lat_probe.py > gpurun_out/lcs_$1_$2.log 2>&1 || { tail -5 gpurun_out/lcs_$1_$2.log; exit 1; }
  tail -1 gpurun_out/lcs_$1_$2.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernel_ms'];print('cfg $1 split $2', d['graph_device_ms'], 'conv6', k['conv6.gemm'], 'conv7', k['conv7.gemm'])"
done
