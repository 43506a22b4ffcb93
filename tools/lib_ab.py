"""A/B of two builds of libdnn_hip.so on one box (compile-time changes that no launch switch
selects): each round runs one child process per library (DNN_HIP_LIB), arms alternating and the
order rotated per round; a child pre-heats the batch-64 plan for --preheat seconds, then times
--iters forwards with per-kernel HIP events (Plan.timing_begin / timing_end).  Prints per arm the
median over rounds of each kernel's mean time and of the forward.

  python tools/lib_ab.py --lib libdnn_hip.so --lib diag/libdnn_hip_old.so [--rounds 4] [--precision fp16]
  python tools/lib_ab.py --env DNN_HIP_X3_IMG=1,0   (plan-time switches: one child per arm)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))
    import torch
    import dnn_hip
    import synth
    import yolo_graph
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(a.batch, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    kw = {"precision": a.precision} if a.precision != "fp32" else {}
    wb, sb = dnn_hip.Plan.memory(a.batch, (416, 416, 3), entries, **kw)
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(sb, dtype=torch.uint8, device=dev)
    plan = dnn_hip.Plan(a.batch, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                        workspace_ptr=sbuf.data_ptr(), **kw)
    x = torch.rand((a.batch, 416, 416, 3), device=dev)
    oshape = (a.batch,) + tuple(plan.out_shape)
    y = torch.empty(oshape, device=dev)
    s = torch.cuda.Stream()
    t0 = time.time()
    while time.time() - t0 < a.preheat:
        for _ in range(10):
            plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
        s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
    e1.record(s)
    s.synchronize()
    fwd = e0.elapsed_time(e1) / a.iters
    plan.timing_begin(a.iters)
    for _ in range(a.iters):
        plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
    ms, cnt = plan.timing_end()
    ker = {k["name"]: m / max(c, 1) for k, m, c in zip(plan.kernels(), ms, cnt)}
    print("RESULT " + json.dumps({"fwd_ms": fwd, "kernels": ker}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--env", default=None, help="VAR=v1,v2,...: arms over an environment variable")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--preheat", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    arms = []  # (name, env overrides)
    if a.env:
        var, vals = a.env.split("=", 1)
        arms = [("%s=%s" % (var, v), {var: v}) for v in vals.split(",")]
    else:
        arms = [(lib, {"DNN_HIP_LIB": lib}) for lib in a.lib]
    res = {name: [] for name, _ in arms}
    for r in range(a.rounds):
        order = arms[r % len(arms):] + arms[:r % len(arms)]
        for lib, over in order:
            env = dict(os.environ, **over)
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(a.iters),
                                  "--preheat", str(a.preheat), "--batch", str(a.batch), "--precision", a.precision],
                                 env=env, capture_output=True, text=True, timeout=600)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT ")]
            if out.returncode != 0 or not line:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(1)
            res[lib].append(json.loads(line[0][7:]))
            print("round", r, lib, "fwd %.4f" % res[lib][-1]["fwd_ms"], flush=True)
    for lib, rs in res.items():
        ks = rs[0]["kernels"].keys()
        med = {k: round(statistics.median(x["kernels"][k] for x in rs), 4) for k in ks}
        print(json.dumps({"arm": lib, "fwd_ms_median": round(statistics.median(x["fwd_ms"] for x in rs), 4),
                          "kernels_ms_median": med}))


if __name__ == "__main__":
    main()
