# A/B: static s_setprio 1 for the x3 patch kernel's second wave half (DNN_HIP_X3PRIO)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3prio; mkdir -p $O; cd $R
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for v in 0 1 0 1; do
DNN_HIP_X3PRIO=$v timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('PRIO=$v', d['value'], {n:round(v['ms'],4) for n,v in k.items() if n[:5] in ('conv4','conv5','conv6','conv7')})"
done
