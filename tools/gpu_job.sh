#!/bin/bash
# One parameterised launcher for GPU-box work (gpurun), replacing the per-experiment job
# scripts of rounds 1-2.  Usage (from the repo root, under gpurun):
#   bash tools/gpu_job.sh TASK [ARGS...]
# Tasks (output under gpurun_out/$OUT, default gpurun_out/job):
#   tests [PYTEST_ARGS...]     pytest -m gpu (extra args passed through, e.g. -k x3)
#   bench [BENCH_ARGS...]      one bench.py line (fp32 forward only unless args say otherwise)
#   ab VAR V1 V2 [BENCH_ARGS]  bench.py --kernels with env VAR=V1, then VAR=V2, then V1 again
#   sweep VAR V1 V2 ...        bench.py --kernels (forward only) for each value of env VAR, then V1 again
#   lat VAR V1 V2 ...          the batch-1 latency plan (latency_b1) for each value of env VAR
#   trace [BENCH_ARGS...]      rocprofv3 --kernel-trace --stats of a short bench run
#   lattrace [BENCH_ARGS...]   kernel trace of the batch-1 latency plan's replays, by (kernel, grid)
#   pmc GROUP [BENCH_ARGS...]  one rocprofv3 --pmc pass: GROUP = fetch | write | sqa | sqb
#   full                       round evidence: tests, default bench line, trace, fetch/write, SQ a/b
#   profiles                   the profile part of the round evidence for the fused fp32 plan
#                              (trace, FETCH/WRITE, SQ a/b), the unfused plan and the fp16 plan
#                              (trace, FETCH/WRITE); tools/summarize_profiles.sh turns it into profiles/
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-job}
mkdir -p "$O"
cd "$R" || exit 1
FAST="--no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --no-fp32-mfma"
# counter passes serialise every dispatch: no pre-heat / sustained windows there (the kernel-trace
# passes keep them, so their durations are the steady-state ones)
NOHEAT="--preheat 0 --sustained 0"

run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > "$O/pytest_gpu.log" 2>&1
  local rc=$?
  grep -E "passed|failed|error" "$O/pytest_gpu.log" | tail -3
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$O/pytest_gpu.log" | head -30; }
  return $rc
}

run_bench() {  # $1 = log name, rest = bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; return 1; }
  tail -1 "$O/$name.log" > "$O/$name.json"
  python - "$O/$name.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("value %.1f img/s  ms/step %.4f  roofline %s" % (d["value"], d["ms_per_step"], {k: d["roofline"].get(k) for k in ("achieved", "frac")}))
k = d.get("kernels")
if k:
    print("  " + "  ".join("%s %.4f" % (n.replace(".gemm", "").replace(".direct", ""), v["ms"]) for n, v in k.items()))
EOF
}

prof() {  # $1 = dir name, $2.. = rocprofv3 options then '--' handled here
  local name=$1; shift
  local opts=()
  while [ "$1" != "--" ]; do opts+=("$1"); shift; done
  shift
  (cd /tmp && timeout -s KILL 300 rocprofv3 "${opts[@]}" -d "$O/$name" -o "$name" --output-format csv -- python3 "$R/bench.py" "$@" > "$O/$name.log" 2>&1) || { tail -5 "$O/$name.log"; return 1; }
}

task=$1; shift
case $task in
  tests) run_tests "$@" ;;
  bench) run_bench bench "$@" ;;
  ab)
    var=$1; v1=$2; v2=$3; shift 3
    export "$var=$v1"; run_bench "ab_$v1" --kernels $FAST "$@" || exit 1
    export "$var=$v2"; run_bench "ab_$v2" --kernels $FAST "$@" || exit 1
    export "$var=$v1"; run_bench "ab_${v1}_again" --kernels $FAST "$@" || exit 1
    ;;
  sweep)
    var=$1; shift
    first=$1
    for v in "$@" "$first"; do
      export "$var=$v"; run_bench "sweep_$v" --kernels $FAST --steps 20 --warmup 3 || exit 1
    done
    ;;
  lat)
    var=$1; shift
    for v in "$@"; do
      export "$var=$v"
      timeout -k 10 400 python bench.py --no-cpu --no-fp16 --no-unfused --no-e2e --no-fp32-mfma --steps 3 --warmup 1 \
        > "$O/lat_$v.log" 2>&1 || { tail -20 "$O/lat_$v.log"; exit 1; }
      tail -1 "$O/lat_$v.log" > "$O/lat_$v.json"
      python - "$O/lat_$v.json" "$var=$v" <<'EOF2'
import json, sys
d = json.loads(open(sys.argv[1]).read())["latency_b1"]
print(sys.argv[2], "graph_device_ms %.4f graph_ms %.4f" % (d["graph_device_ms"], d["graph_ms"]))
print("  " + "  ".join("%s %.4f" % (n, v) for n, v in d["kernel_ms"].items()))
EOF2
    done
    ;;
  lattrace)
    prof lattrace --kernel-trace -- --steps 1 --warmup 1 --no-cpu --no-fp16 --no-unfused --no-e2e --no-fp32-mfma "$@" || exit 1
    python tools/trace_by_grid.py $(find "$O/lattrace" -name "*kernel_trace.csv") --min-count 100 > "$O/lattrace.txt" && cat "$O/lattrace.txt"
    ;;
  trace) prof trace --kernel-trace --stats -- --steps 10 --warmup 3 $FAST "$@" ;;
  pmc)
    group=$1; shift
    case $group in
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE" ;;
      sqa) C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" ;;
      sqb) C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" ;;
      *) echo "unknown pmc group $group"; exit 2 ;;
    esac
    # --gather outputs: no postprocess kernels on the side stream, so no other kernel runs
    # beside a profiled dispatch (GRBM_GUI_ACTIVE and the SQ counters sample the whole GPU:
    # a concurrent postprocess inflated round 2's conv4 row 5x)
    prof "pmc_$group" --pmc $C -- --steps 3 --warmup 1 $FAST $NOHEAT --gather outputs "$@"
    ;;
  profiles)
    P="--gather outputs"
    # (the traces run with --gather outputs too: no postprocess kernel beside conv0 / conv1)
    prof fused_trace --kernel-trace --stats -- --steps 10 --warmup 3 $FAST $P || exit 1
    prof fused_fetch --pmc FETCH_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P || exit 1
    prof fused_write --pmc WRITE_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P || exit 1
    for g in sqa sqb; do bash "$0" pmc $g || exit 1; done
    export DNN_HIP_FUSE=0
    prof unf_trace --kernel-trace --stats -- --steps 10 --warmup 3 $FAST $P || exit 1
    prof unf_fetch --pmc FETCH_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P || exit 1
    prof unf_write --pmc WRITE_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P || exit 1
    unset DNN_HIP_FUSE
    prof f16_trace --kernel-trace --stats -- --steps 10 --warmup 3 $FAST $P --precision fp16 || exit 1
    prof f16_fetch --pmc FETCH_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P --precision fp16 || exit 1
    prof f16_write --pmc WRITE_SIZE -- --steps 3 --warmup 1 $FAST $NOHEAT $P --precision fp16 || exit 1
    echo PROFILESOK
    ;;
  full)
    run_tests || exit 1
    run_bench bench --kernels || exit 1
    prof trace --kernel-trace --stats -- --steps 10 --warmup 3 $FAST || exit 1
    for g in fetch write sqa sqb; do
      bash "$0" pmc $g || exit 1
    done
    echo FULLOK
    ;;
  *) echo "unknown task $task"; exit 2 ;;
esac
