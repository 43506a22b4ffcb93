# fp16 plan (BASELINE config 5) profile: kernel trace + stats, FETCH/WRITE passes, SQ/GRBM passes.
# Output under gpurun_out/f16_*; summarise with tools/prof_summary.py --fp16 / tools/pmc_table.py --fp16.
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp
B="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --precision fp16"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f16_trace -o trace --output-format csv -- $B > $R/gpurun_out/f16_trace.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/f16_fetch -o fetch --output-format csv -- $B > $R/gpurun_out/f16_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/f16_write -o write --output-format csv -- $B > $R/gpurun_out/f16_write.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/f16_sqa -o a --output-format csv -- $B > $R/gpurun_out/f16_sqa.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $R/gpurun_out/f16_sqb -o b --output-format csv -- $B > $R/gpurun_out/f16_sqb.log 2>&1 || exit 1
echo F16PROFOK
