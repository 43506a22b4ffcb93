"""Single-frame latency plan (BASELINE config 2) under different HIP runtime environments: one child
process per arm (the runtime reads its environment at start-up), arms alternating for --rounds
rounds.  A child measures what bench.py's latency_b1 measures: the median wall time of a
synchronised eager forward and of a synchronised graph replay, and the device time of back-to-back
graph replays (HIP events).

  python tools/lat_env.py --env="HIP_FORCE_DEV_KERNARG=0;HIP_FORCE_DEV_KERNARG=1" [--rounds 3]
  (arms split on ';', each a comma-separated list of VAR=VALUE, '-' for the unchanged environment)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(iters):
    sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))
    import torch
    import dnn_hip
    import synth
    import yolo_graph
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    g1, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(1, 416, 416, 3))
    entries = dnn_hip.lower_graph(g1)
    wb, sb = dnn_hip.Plan.memory(1, (416, 416, 3), entries, latency=True)
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
    p1 = dnn_hip.Plan(1, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                      workspace_ptr=sbuf.data_ptr(), latency=True)
    x = torch.rand((1, 416, 416, 3), device=dev)
    y = torch.empty((1, 13, 13, 125), device=dev)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    out = {}
    t_end = time.time() + 1.0
    while time.time() < t_end:  # pre-heat
        for _ in range(20):
            p1.run_device(1, x.data_ptr(), y.data_ptr(), sp)
        s.synchronize()
    for mode in ("eager", "graph"):
        run = p1.run_device if mode == "eager" else p1.run_graph
        for _ in range(20):
            run(1, x.data_ptr(), y.data_ptr(), sp)
        s.synchronize()
        t = []
        for _ in range(iters):
            t0 = time.perf_counter()
            run(1, x.data_ptr(), y.data_ptr(), sp)
            s.synchronize()
            t.append(time.perf_counter() - t0)
        out[mode + "_ms"] = round(statistics.median(t) * 1e3, 4)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(100):
            p1.run_graph(1, x.data_ptr(), y.data_ptr(), sp)
        e1.record(s)
    s.synchronize()
    out["graph_device_ms"] = round(e0.elapsed_time(e1) / 100, 4)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(100):
            p1.run_device(1, x.data_ptr(), y.data_ptr(), sp)
        e1.record(s)
    s.synchronize()
    out["eager_device_ms"] = round(e0.elapsed_time(e1) / 100, 4)
    p1.timing_begin(100)
    for _ in range(100):
        p1.run_device(1, x.data_ptr(), y.data_ptr(), sp)
    ms, cnt = p1.timing_end()
    out["kernels_us"] = {k["name"]: round(1e3 * m / max(c, 1), 2) for k, m, c in zip(p1.kernels(), ms, cnt)}
    print(json.dumps(out), flush=True)
    p1.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="-")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.iters)
        return
    arms = a.env.split(";")
    res = {arm: [] for arm in arms}
    for r in range(a.rounds):
        order = arms[r % len(arms):] + arms[:r % len(arms)]
        for arm in order:
            env = dict(os.environ)
            if arm != "-":
                for kv in arm.split(","):
                    k, v = kv.split("=", 1)
                    env[k] = v
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(a.iters)],
                               env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-2000:])
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[arm].append(d)
            print("round", r, arm, d, flush=True)
    for arm, v in res.items():
        med = {k: statistics.median(x[k] for x in v) for k in v[0] if k != "kernels_us"}
        med["kernels_us"] = {k: statistics.median(x["kernels_us"][k] for x in v) for k in v[0]["kernels_us"]}
        print(json.dumps({"arm": arm, **med}), flush=True)


if __name__ == "__main__":
    main()
