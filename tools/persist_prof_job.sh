# tests touching the GEMM variants, then a same-box rocprof A/B of the persistent short-K GEMM
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pab; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "latency or splitk or persistent or yolo or implicit or buffer_dma or fused" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
F="--no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --steps 10 --warmup 3"
for on in 1 0; do
DNN_HIP_PERSIST=$on timeout -k 10 200 rocprofv3 --kernel-trace -d $O/p$on -o trace --output-format csv -- python3 $R/bench.py $F > $O/p$on.log 2>&1 || exit 1
done
cd $R; for on in 1 0; do python3 tools/prof_summary.py --skip 3 --trace $O/p$on/trace_kernel_trace.csv 2>&1 | grep -E "^conv" | sed "s/^/persist=$on /" | cut -c1-60; done
