# all GPU tests, then the fp32 bench A/B: x3 default vs DNN_HIP_X3=0 (per-kernel times)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3f; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "normwise|FAIL|Error|^E " $O/pytest.log | tail -30; exit 1; }
grep -E "normwise|passed|failed" $O/pytest.log | tail -12
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for a in DNN_HIP_X3=1 DNN_HIP_X3=0; do
env $a timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('$a', d['value'], {n:v['ms'] for n,v in k.items()})"
done
