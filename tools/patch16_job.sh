# fp16 patch conv (conv6/conv7): tests, then the fp16 bench line with per-kernel times
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fp16 or shape_only" > gpurun_out/pytest_p16.log 2>&1 || { tail -40 gpurun_out/pytest_p16.log; exit 1; }
tail -2 gpurun_out/pytest_p16.log
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels --precision fp16"
for on in 1 0; do export DNN_HIP_PATCH16=$on;
DNN_HIP_PATCH16=$on timeout -k 10 120 python bench.py $F > gpurun_out/p16b_$on.log 2>&1 || { tail -5 gpurun_out/p16b_$on.log; exit 1; }
tail -1 gpurun_out/p16b_$on.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('patch16=$on', d['value'], {n:(v['ms'],v['tflops']) for n,v in k.items() if n in ('conv5.gemm','conv6.gemm','conv7.gemm')})"
done
