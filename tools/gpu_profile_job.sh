export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --kernels > gpurun_out/bench6.log 2>&1 || { tail -20 gpurun_out/bench6.log; exit 1; }
cd /tmp
F="--no-cpu --no-latency --no-fp16 --no-unfused --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1c -o trace --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $F > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_c -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $F > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_c -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $F > $R/gpurun_out/pmc_write.log 2>&1 || exit 1
# the unfused plan (explicit im2col + GEMM + separate pools): im2col HBM GB/s and traffic
export DNN_HIP_FUSE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_unf -o trace --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 $F > $R/gpurun_out/prof_unf.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_unf -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $F > $R/gpurun_out/pmc_fetch_unf.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_unf -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $F > $R/gpurun_out/pmc_write_unf.log 2>&1 || exit 1
echo ALLOK
