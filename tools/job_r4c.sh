set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
for d in ${DIAGS:-16 17 18 24 26 27}; do
  DNN_HIP_LIB=diag/libdnn_hip_d$d.so timeout -k 10 200 python tools/x3_ab.py --rounds 2 --preheat 3 > $O/d$d.log 2>&1 || { tail -20 $O/d$d.log; exit 1; }
  python - $O/d$d.log $d <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
a = list(d["arms"].values())[0]
c = a.get("clock_last_round", {})
print("d%s conv6 %.4f conv7 %.4f  ghz %.3f  loop_us %.1f max %.1f  Mcyc %.4f [%.4f..%.4f] span %.1f" % (sys.argv[2],
      a["kernels_ms_median"]["conv6.gemm"], a["kernels_ms_median"]["conv7.gemm"], c.get("median_ghz", 0),
      c.get("median_loop_us", 0), c.get("max_loop_us", 0), c.get("mcycles_median", 0), c.get("mcycles_min", 0),
      c.get("mcycles_max", 0), c.get("span_us", 0)))
PY
done
