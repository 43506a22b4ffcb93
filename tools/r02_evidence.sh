# Summarise a round-2 profile job's output (gpurun_out/$1, tools/r02_profile_job.sh) into profiles/.
set -e
D=gpurun_out/${1:-r02b}; P=profiles
python3 tools/prof_summary.py --skip 3 --trace $D/fused_trace/trace_kernel_trace.csv --fetch $D/fused_fetch/fetch_counter_collection.csv --write $D/fused_write/write_counter_collection.csv --note "round 2: fused fp32 plan (x3 conv6/conv7), bench.py --steps 10 --warmup 3 (trace), --steps 3 --warmup 1 (FETCH_SIZE, WRITE_SIZE passes), MI355X" --out $P/pmc_summary.json
python3 tools/prof_summary.py --skip 3 --unfused --trace $D/unf_trace/trace_kernel_trace.csv --fetch $D/unf_fetch/fetch_counter_collection.csv --write $D/unf_write/write_counter_collection.csv --note "round 2: DNN_HIP_FUSE=0 plan (explicit im2col + GEMM, separate pools), MI355X" --out $P/pmc_summary_unfused.json
python3 tools/prof_summary.py --skip 3 --fp16 --trace $D/f16_trace/trace_kernel_trace.csv --fetch $D/f16_fetch/fetch_counter_collection.csv --write $D/f16_write/write_counter_collection.csv --note "round 2: fp16 plan (BASELINE config 5), MI355X" --out $P/pmc_summary_fp16.json
cp $D/fused_trace/trace_kernel_stats.csv $P/r02_rocprof_kernel_stats.csv
cp $D/unf_trace/trace_kernel_stats.csv $P/r02_rocprof_kernel_stats_unfused.csv
cp $D/f16_trace/trace_kernel_stats.csv $P/r02_rocprof_kernel_stats_fp16.csv
tail -1 $D/bench.log > $P/r02_bench.json
python3 tools/pmc_table.py $D/sq_a/*counter_collection.csv $D/sq_b/*counter_collection.csv --out $P/r02_sq_counters_fp32.json > /dev/null
echo done
