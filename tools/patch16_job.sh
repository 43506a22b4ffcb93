# fp16 patch conv (conv6/conv7): tests for both MFMA shapes, then the fp16 bench line with
# per-kernel times for each shape (DNN_HIP_P16MF) and the glds kernel (DNN_HIP_PATCH16=0)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for mf in 16 32; do
DNN_HIP_P16MF=$mf timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fp16 or shape_only" > gpurun_out/pytest_p16_$mf.log 2>&1 || { tail -40 gpurun_out/pytest_p16_$mf.log; exit 1; }
tail -2 gpurun_out/pytest_p16_$mf.log
done
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels --precision fp16"
for arm in "1 16" "1 32" "0 16" "1 16"; do set -- $arm
DNN_HIP_PATCH16=$1 DNN_HIP_P16MF=$2 timeout -k 10 120 python bench.py $F > gpurun_out/p16b_$1_$2.log 2>&1 || { tail -5 gpurun_out/p16b_$1_$2.log; exit 1; }
tail -1 gpurun_out/p16b_$1_$2.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('patch16=$1 mf=$2', d['value'], {n:(v['ms'],v['tflops']) for n,v in k.items() if n in ('conv5.gemm','conv6.gemm','conv7.gemm')})"
done
