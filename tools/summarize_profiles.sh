#!/bin/bash
# Turn a `tools/gpu_job.sh profiles` run (gpurun_out/$2) and its bench line
# (gpurun_out/$3/bench.json, from `tools/gpu_job.sh bench --kernels`) into the committed
# round evidence under profiles/:  bash tools/summarize_profiles.sh r03 prof bench
set -e
R=$1; D=gpurun_out/$2; B=gpurun_out/${3:-$2}; P=profiles
python3 tools/prof_summary.py --skip 3 --trace $D/fused_trace/fused_trace_kernel_trace.csv \
  --fetch $D/fused_fetch/fused_fetch_counter_collection.csv --write $D/fused_write/fused_write_counter_collection.csv \
  --note "round ${R#r}: fused fp32 plan (x3 conv1-conv8), bench.py --steps 10 --warmup 3 (trace), --steps 3 --warmup 1 --gather outputs (FETCH_SIZE, WRITE_SIZE passes), MI355X" \
  --out $P/pmc_summary.json
python3 tools/prof_summary.py --skip 3 --unfused --trace $D/unf_trace/unf_trace_kernel_trace.csv \
  --fetch $D/unf_fetch/unf_fetch_counter_collection.csv --write $D/unf_write/unf_write_counter_collection.csv \
  --note "round ${R#r}: DNN_HIP_FUSE=0 plan (explicit im2col + GEMM, separate pools), MI355X" --out $P/pmc_summary_unfused.json
python3 tools/prof_summary.py --skip 3 --fp16 --trace $D/f16_trace/f16_trace_kernel_trace.csv \
  --fetch $D/f16_fetch/f16_fetch_counter_collection.csv --write $D/f16_write/f16_write_counter_collection.csv \
  --note "round ${R#r}: fp16 plan (BASELINE config 5), MI355X" --out $P/pmc_summary_fp16.json
# the bench line of the SAME gpurun call (same box) beside the trace: its HIP-event duration of the
# dominant kernel, fraction and img/s (bench.py reports them as roofline.rocprof_same_box)
python3 - "$B/bench.json" "$P/pmc_summary.json" <<'EOF'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = json.load(open(sys.argv[2]))
r = b["roofline"]
p["same_box"] = {"images_per_s": b["value"], "ms_per_step": b["ms_per_step"], "dominant_kernel": r["kernel"],
                 "dominant_event_ms": r["avg_launch_ms"], "event_frac": r["frac"],
                 "sclk_ghz": r.get("sclk_ghz"), "sclk_ghz_timed_region": r.get("sclk_ghz_timed_region"),
                 "event_frac_at_measured_clock": r.get("frac_at_measured_clock"),
                 "note": "bench.py line of the same gpurun call (same box) as this trace"}
json.dump(p, open(sys.argv[2], "w"), indent=1)
EOF
cp $D/fused_trace/fused_trace_kernel_stats.csv $P/${R}_rocprof_kernel_stats.csv
cp $D/unf_trace/unf_trace_kernel_stats.csv $P/${R}_rocprof_kernel_stats_unfused.csv
cp $D/f16_trace/f16_trace_kernel_stats.csv $P/${R}_rocprof_kernel_stats_fp16.csv
cp $B/bench.json $P/${R}_bench.json
# the committed bench line's rocprof fields from THIS call's trace and PMC passes (bench.py read the
# previous round's summary when it ran): same box, same build
python3 - "$P/${R}_bench.json" "$P/pmc_summary.json" <<'PYEOF'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = json.load(open(sys.argv[2]))
r = b["roofline"]
k = p["kernels"].get(r["kernel"], {})
if k.get("avg_us"):
    mult = r["achieved"] * r["avg_launch_ms"] / 1e3 / (r["flops_per_launch"] / 1e12) if r.get("flops_per_launch") else 6.0
    r["rocprof_avg_launch_ms"] = round(k["avg_us"] / 1e3, 4)
    r["rocprof_frac"] = round(mult * r["flops_per_launch"] / (k["avg_us"] / 1e6) / 1e12 / r["peak"], 4)
    r["rocprof_same_box"] = p.get("same_box")
    r["rocprof_source"] = "profiles/pmc_summary.json: rocprofv3 --kernel-trace of bench.py in the same gpurun call (same box) as this line"
if k.get("hbm_bytes_per_launch"):
    r["traffic"] = k["hbm_bytes_per_launch"]
    if r.get("algorithmic_bytes"):
        r["traffic_over_algorithmic"] = round(k["hbm_bytes_per_launch"] / r["algorithmic_bytes"], 2)
open(sys.argv[1], "w").write(json.dumps(b) + "\n")
PYEOF
python3 tools/pmc_table.py $D/pmc_sqa/*counter_collection.csv $D/pmc_sqb/*counter_collection.csv \
  --out $P/${R}_sq_counters_fp32.json > /dev/null
echo done
