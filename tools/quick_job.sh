# quick GPU check: the GPU test suite, then the bench's main line (no extras)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels > gpurun_out/bq.log 2>&1 || { tail -20 gpurun_out/bq.log; exit 1; }
tail -1 gpurun_out/bq.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['per_rank']);print({k:v['ms'] for k,v in d['kernels'].items()})"
