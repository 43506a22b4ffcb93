# fp16 tile-config sweep: DNN_HIP_CFG16 variants as arguments ("-" = chooser default)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
i=0
for c in "$@"; do
  i=$((i+1))
  if [ "$c" = "-" ]; then unset DNN_HIP_CFG16; else export DNN_HIP_CFG16="$c"; fi
  timeout -k 10 200 python bench.py --precision fp16 --steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels > gpurun_out/cfg16_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/cfg16_$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
done
