# SQ / GRBM counter passes over a short bench.py run (one counter group per pass, no traces
# combined with --pmc).  Output under gpurun_out/sq_*.
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --precision ${PREC:-fp32}"
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/sq_trace -o trace --output-format csv -- $B > $R/gpurun_out/sq_trace.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/sq_a -o a --output-format csv -- $B > $R/gpurun_out/sq_a.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $R/gpurun_out/sq_b -o b --output-format csv -- $B > $R/gpurun_out/sq_b.log 2>&1 || exit 1
echo SQOK
