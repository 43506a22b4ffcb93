# persistent short-K GEMM: bit-exactness tests, then A/B on the bench line
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "persistent or implicit_gemm or yolo_batch64 or buffer_dma" > gpurun_out/pytest_persist.log 2>&1 || { tail -40 gpurun_out/pytest_persist.log; exit 1; }
tail -2 gpurun_out/pytest_persist.log
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for on in 1 0; do
  DNN_HIP_PERSIST=$on timeout -k 10 120 python bench.py $F > gpurun_out/persist_$on.log 2>&1 || { tail -5 gpurun_out/persist_$on.log; exit 1; }
  tail -1 gpurun_out/persist_$on.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('persist=$on', d['value'], {n:v['ms'] for n,v in k.items() if n in ('conv2.gemm','conv3.gemm','conv4.gemm')})"
done
for w in 2; do
  DNN_HIP_PERSIST_WGS=$w timeout -k 10 120 python bench.py $F > gpurun_out/persist_w$w.log 2>&1 || { tail -5 gpurun_out/persist_w$w.log; exit 1; }
  tail -1 gpurun_out/persist_w$w.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('wgs=$w', d['value'], {n:v['ms'] for n,v in k.items() if n in ('conv2.gemm','conv3.gemm','conv4.gemm')})"
done
