# A/B of an env switch on the bench main line: default vs $ABVAR=0, alternated twice
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
run() { timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels > gpurun_out/ab_$1.log 2>&1 || exit 1;
  tail -1 gpurun_out/ab_$1.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items() if k in ('conv0.direct','conv1.patch','conv2.gemm','conv3.gemm','conv4.gemm')})"; }
run def1; env $ABVAR=0 bash -c true; export $ABVAR=0; run off1; unset $ABVAR; run def2; export $ABVAR=0; run off2
