# explicit-im2col (unfused plan) tests and a block-size sweep of the VEC kernel
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "im2col or implicit_gemm or fused_conv" > gpurun_out/pytest_im2col.log 2>&1 || { tail -40 gpurun_out/pytest_im2col.log; exit 1; }
tail -2 gpurun_out/pytest_im2col.log
F="--steps 3 --warmup 1 --no-cpu --no-latency --no-fp16 --no-e2e"
for fl in 8192 4096 8192 4096; do
  DNN_HIP_IM2COL_FLOATS=$fl timeout -k 10 120 python bench.py $F > gpurun_out/im2col_$fl.log 2>&1 || { tail -5 gpurun_out/im2col_$fl.log; exit 1; }
  tail -1 gpurun_out/im2col_$fl.log | python -c "import json,sys;d=json.loads(sys.stdin.read())['unfused'];print('floats $fl', d['im2col_total'], {k:(v['ms'],v['gbs']) for k,v in d['im2col'].items()})"
done
