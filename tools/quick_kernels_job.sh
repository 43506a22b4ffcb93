# GPU tests (pattern K), then the fp32 bench per-kernel table twice
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/qk; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for a in 1 2; do
timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print(d['value'], {n:v['ms'] for n,v in k.items()})"
done
