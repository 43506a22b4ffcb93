set -o pipefail
mkdir -p gpurun_out/diag
for L in ${LIBS:-libdnn_hip.so}; do
  n=$(basename $L .so)
  DNN_HIP_LIB=$L timeout -k 10 300 python bench.py --kernels --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --no-fp32-mfma --steps 20 --warmup 3 > gpurun_out/diag/$n.log 2>&1 || { tail -5 gpurun_out/diag/$n.log; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/diag/$n.log').read().strip().split('\n')[-1]); k=d['kernels']
print('$n', ' '.join('%s %.4f'%(a.split('.')[0],k[a]['ms']) for a in k))"
done
