# fp16 folded epilogue + shape-only plan: tests, then the fp16 bench line
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fp16 or shape_only or buffer_dma or dist" > gpurun_out/pytest_f16.log 2>&1 || { tail -40 gpurun_out/pytest_f16.log; exit 1; }
tail -2 gpurun_out/pytest_f16.log
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels --precision fp16"
timeout -k 10 120 python bench.py $F > gpurun_out/f16b.log 2>&1 || { tail -5 gpurun_out/f16b.log; exit 1; }
tail -1 gpurun_out/f16b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print(d['value'], {n:v['ms'] for n,v in k.items()})"
