# A/B of the bench step: plain process vs under torch.distributed.run (RCCL group, world 1),
# detection gather modes sized / fixed; then the distributed GPU tests
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
F="--steps 50 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e"
show() { tail -1 $1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$2', d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['dist_backend'],d['per_rank'])"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { tail -30 gpurun_out/pytest_dist.log; exit 1; }
tail -1 gpurun_out/pytest_dist.log
for m in sized fixed; do
DNN_BENCH_GATHER_MODE=$m timeout -k 10 200 python bench.py $F > gpurun_out/ab_plain.log 2>&1 || exit 1
show gpurun_out/ab_plain.log plain_$m
DNN_BENCH_GATHER_MODE=$m timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py $F > gpurun_out/ab_trun.log 2>&1 || exit 1
show gpurun_out/ab_trun.log torchrun_$m
done
