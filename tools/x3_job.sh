# fp32 x3 conv (conv6/conv7 on exact bf16 splits): parity tests, then the fp32 bench line with
# per-kernel times with the x3 conv (default) and without it (DNN_HIP_X3=0)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -k "x3" > gpurun_out/pytest_x3.log 2>&1 || { grep -E "err|PASS|FAIL|Error" gpurun_out/pytest_x3.log | tail -30; exit 1; }
grep -E "normwise|passed|failed" gpurun_out/pytest_x3.log | tail -8
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for x3 in 1 0; do
DNN_HIP_X3=$x3 timeout -k 10 120 python bench.py $F > gpurun_out/x3b_$x3.log 2>&1 || { tail -5 gpurun_out/x3b_$x3.log; exit 1; }
tail -1 gpurun_out/x3b_$x3.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('x3=$x3', d['value'], {n:(v['ms'],v['tflops']) for n,v in k.items() if n in ('pool5','conv5.gemm','conv6.gemm','conv7.gemm','conv8.gemm')})"
done
