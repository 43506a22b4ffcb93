export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
F="--steps 10 --warmup 2 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels --precision fp16"
for d in 0 1 2 3; do
DNN_HIP_P16DBG=$d timeout -k 10 120 python bench.py $F > gpurun_out/p16d_$d.log 2>&1 || { tail -5 gpurun_out/p16d_$d.log; exit 1; }
tail -1 gpurun_out/p16d_$d.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('dbg=$d', {n:(v['ms'],v['tflops']) for n,v in k.items() if n in ('conv6.gemm','conv7.gemm')})"
done
