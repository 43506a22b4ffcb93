# round-2 evidence: GPU tests, the default bench line, rocprof kernel trace + stats and the
# FETCH/WRITE PMC passes of the fused fp32, unfused fp32 and fp16 plans, SQ counter passes
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${PROF_DIR:-r02}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --kernels > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
cd /tmp
F="--no-cpu --no-latency --no-fp16 --no-unfused --no-e2e"
B="python3 $R/bench.py --steps 10 --warmup 3 $F"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fused_trace -o trace --output-format csv -- $B > $O/fused_trace.log 2>&1 || exit 1
B="python3 $R/bench.py --steps 3 --warmup 1 $F"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/fused_fetch -o fetch --output-format csv -- $B > $O/fused_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/fused_write -o write --output-format csv -- $B > $O/fused_write.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq_a -o a --output-format csv -- $B > $O/sq_a.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq_b -o b --output-format csv -- $B > $O/sq_b.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/sq_trace -o trace --output-format csv -- $B > $O/sq_trace.log 2>&1 || exit 1
export DNN_HIP_FUSE=0
B="python3 $R/bench.py --steps 10 --warmup 3 $F"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/unf_trace -o trace --output-format csv -- $B > $O/unf_trace.log 2>&1 || exit 1
B="python3 $R/bench.py --steps 3 --warmup 1 $F"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/unf_fetch -o fetch --output-format csv -- $B > $O/unf_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/unf_write -o write --output-format csv -- $B > $O/unf_write.log 2>&1 || exit 1
unset DNN_HIP_FUSE
B="python3 $R/bench.py --steps 10 --warmup 3 $F --precision fp16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f16_trace -o trace --output-format csv -- $B > $O/f16_trace.log 2>&1 || exit 1
B="python3 $R/bench.py --steps 3 --warmup 1 $F --precision fp16"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/f16_fetch -o fetch --output-format csv -- $B > $O/f16_fetch.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/f16_write -o write --output-format csv -- $B > $O/f16_write.log 2>&1 || exit 1
echo R02OK
