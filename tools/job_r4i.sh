set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
for d in ${DIAGS:-c0d0 c0d1 c0d2 c0d4 c0d6}; do
  DNN_HIP_LIB=diag/libdnn_hip_$d.so timeout -k 10 200 python tools/x3_ab.py --rounds 3 --preheat 3 --kernels conv0,conv1 > $O/$d.log 2>&1 || { tail -20 $O/$d.log; exit 1; }
  python - $O/$d.log $d <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
a = list(d["arms"].values())[0]
print(sys.argv[2], "fwd %.4f" % a["fwd_ms_median"], " ".join("%s %.4f" % (k, v) for k, v in a["kernels_ms_median"].items()))
PY
done
