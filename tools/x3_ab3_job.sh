# bench per-kernel A/B of ARMS (env settings) in one call, the first arm again at the end
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3ab3; mkdir -p $O; cd $R
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for a in $ARMS ${ARMS%% *}; do
env $a timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('$a', d['value'], {n:v['ms'] for n,v in k.items() if n[:5] in ('conv3','conv4','pool4','conv5','pool5')})"
done
