# x3 patch-kernel variants (DNN_HIP_X3V 0..2, default 1): bitwise output equality vs arm 0, the x3 parity
# tests per arm, then a per-kernel bench A/B (arm 0 again at the end)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3v; mkdir -p $O; cd $R
for v in 0 1 2; do
DNN_HIP_X3V=$v timeout -k 10 120 python tools/x3v_out.py $O/out$v.npy > $O/out$v.log 2>&1 || { tail -5 $O/out$v.log; exit 1; }
done
python -c "
import numpy as np
a=np.load('$O/out0.npy')
for v in (1,2):
    b=np.load('$O/out%d.npy'%v); print('arm',v,'bit-equal to arm 0:', a.tobytes()==b.tobytes(), float(np.abs(a-b).max()))
"
for v in 0 2; do
DNN_HIP_X3V=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k x3 > $O/pt$v.log 2>&1 || { tail -20 $O/pt$v.log; exit 1; }
tail -1 $O/pt$v.log
done
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for v in 1 0 2 1; do
DNN_HIP_X3V=$v timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('X3V=$v', d['value'], {n:round(v['ms'],4) for n,v in k.items() if n[:5] in ('conv4','conv5','conv6','conv7')})"
done
