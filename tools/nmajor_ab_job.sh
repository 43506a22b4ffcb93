# A/B of the N-major tile order (DNN_HIP_NMAJOR) on the fp16 and fp32 plans
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for prec in fp16 fp32; do for nm in 0 1 0 1; do
  DNN_HIP_NMAJOR=$nm timeout -k 10 120 python bench.py $F --precision $prec > gpurun_out/nm_${prec}_$nm.log 2>&1 || { tail -5 gpurun_out/nm_${prec}_$nm.log; exit 1; }
  tail -1 gpurun_out/nm_${prec}_$nm.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('$prec nmajor=$nm', d['value'], {n:v['ms'] for n,v in k.items() if n in ('conv4.gemm','conv5.gemm','conv6.gemm','conv7.gemm')})"
done; done
