"""In-process A/B of single-frame latency plans (BASELINE config 2): one plan per arm, each built
with the arm's environment (switches read at plan build, e.g. DNN_HIP_CFG / DNN_HIP_SPLIT, take
effect), captured as a HIP graph, then the arms' graph replays interleaved round by round.

  python tools/lat_ab.py --env "DNN_HIP_SPLIT=;2304:4" [--rounds 8] [--reps 50]   (arm values split on ";")

Prints per arm the median over rounds of the device time of one graph replay (HIP events around
`reps` back-to-back replays, bench.py latency_b1's `graph_device_ms`), the per-kernel HIP-event
times of eager runs, and the normwise difference of the arm's output from the first arm's."""
import argparse
import ctypes
import json
import os
import statistics
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))

import torch  # noqa: E402

import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402


def ktile_stamps(lib):
    """X3DIAG bit 256 builds: conv3x3_x3_ktile_kernel's per-workgroup s_memrealtime stamps (100 MHz)
    of the last launch of each shape: start skew, patch, MFMA and epilogue phases (us)."""
    fn = getattr(lib, "dnn_ktile_diag_stamps", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (4 * 1024))()
    if fn(buf, 1024) != 0:
        return None
    out = {}
    for name, base in (("w26", 0), ("w13", 512)):
        rows = [buf[4 * w:4 * w + 4] for w in range(base, base + 512) if buf[4 * w] and buf[4 * w + 3] >= buf[4 * w]]
        if not rows:
            continue
        t0 = min(r[0] for r in rows)
        med = lambda f: round(statistics.median(f(r) for r in rows) / 100.0, 2)  # noqa: E731
        out[name] = {"workgroups": len(rows), "start_skew_max": round(max(r[0] - t0 for r in rows) / 100.0, 2),
                     "patch": med(lambda r: r[1] - r[0]), "mfma": med(lambda r: r[2] - r[1]),
                     "epilogue": med(lambda r: r[3] - r[2]), "span": round((max(r[3] for r in rows) - t0) / 100.0, 2)}
    return out


def lat_stamps(lib):
    """X3DIAG bit 512 builds: conv3x3_x3_lat_kernel's per-workgroup s_memrealtime stamps of its last
    launch (conv7): start skew, patch, MFMA and store phases (us)."""
    fn = getattr(lib, "dnn_lat_diag_stamps", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (4 * 1024))()
    if fn(buf, 1024) != 0:
        return None
    rows = [buf[4 * w:4 * w + 4] for w in range(1024) if buf[4 * w] and buf[4 * w + 3] >= buf[4 * w]]
    if not rows:
        return None
    t0 = min(r[0] for r in rows)
    med = lambda f: round(statistics.median(f(r) for r in rows) / 100.0, 2)  # noqa: E731
    mx = lambda f: round(max(f(r) for r in rows) / 100.0, 2)  # noqa: E731
    return {"workgroups": len(rows), "start_skew_max": mx(lambda r: r[0] - t0),
            "patch": med(lambda r: r[1] - r[0]), "patch_max": mx(lambda r: r[1] - r[0]),
            "mfma": med(lambda r: r[2] - r[1]), "mfma_max": mx(lambda r: r[2] - r[1]),
            "store": med(lambda r: r[3] - r[2]), "span": mx(lambda r: r[3] - t0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", action="append", default=[], help="VAR=v1;v2;... (arms; an empty value unsets)")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    arms = [{}]
    for spec in a.env:
        var, vals = spec.split("=", 1)
        arms = [dict(x, **{var: v}) for x in arms for v in vals.split(";")]
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    g1, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(1, 416, 416, 3))
    entries = dnn_hip.lower_graph(g1)
    x = torch.rand((1, 416, 416, 3), generator=torch.Generator(device=dev).manual_seed(3), device=dev)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    base = dict(os.environ)
    keys = {k for arm in arms for k in arm}

    def set_arm(arm):
        for k in keys:
            if k in base:
                os.environ[k] = base[k]
            else:
                os.environ.pop(k, None)
        for k, v in arm.items():
            if v:
                os.environ[k] = v

    plans = []
    for arm in arms:
        set_arm(arm)
        wb, sb = dnn_hip.Plan.memory(1, (416, 416, 3), entries, latency=True)
        wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
        sbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
        p = dnn_hip.Plan(1, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                         workspace_ptr=sbuf.data_ptr(), latency=True)
        y = torch.empty((1, 13, 13, 125), device=dev)
        for _ in range(5):
            p.run_graph(1, x.data_ptr(), y.data_ptr(), sp)
        s.synchronize()
        plans.append({"arm": arm, "plan": p, "y": y, "bufs": (wbuf, sbuf), "graph": [], "k": {}})
        print(json.dumps(arm), "plan:\n" + p.describe(), flush=True)
    y0 = plans[0]["y"].clone()
    for r in range(a.rounds):
        order = plans[r % len(plans):] + plans[:r % len(plans)]
        if r % 2:
            order = order[::-1]
        for d in order:
            set_arm(d["arm"])
            p = d["plan"]
            for _ in range(10):
                p.run_graph(1, x.data_ptr(), d["y"].data_ptr(), sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                for _ in range(a.reps):
                    p.run_graph(1, x.data_ptr(), d["y"].data_ptr(), sp)
                e1.record(s)
            s.synchronize()
            d["graph"].append(e0.elapsed_time(e1) / a.reps)
            p.timing_begin(20)
            for _ in range(20):
                p.run_device(1, x.data_ptr(), d["y"].data_ptr(), sp)
            ms, cnt = p.timing_end()
            for k, m, c in zip(p.kernels(), ms, cnt):
                d["k"].setdefault(k["name"], []).append(m / max(c, 1))
            kt = ktile_stamps(p.lib)
            if kt:
                d["ktile"] = kt
            lt = lat_stamps(p.lib)
            if lt:
                d["lat"] = lt
    # a tail of graph replays of arm 0 (a kernel trace of this run ends with whole replays:
    # tools/trace_timeline.py)
    d = plans[0]
    set_arm(d["arm"])
    for _ in range(a.reps):
        d["plan"].run_graph(1, x.data_ptr(), d["y"].data_ptr(), sp)
    s.synchronize()
    out = {}
    for d in plans:
        y = d["y"]
        err = float((y - y0).norm() / y0.norm())
        rec = {"graph_device_ms_median": round(statistics.median(d["graph"]), 4),
               "graph_device_ms_min": round(min(d["graph"]), 4),
               "kernels_ms_median": {k: round(statistics.median(v), 4) for k, v in d["k"].items()},
               "normwise_vs_arm0": err}
        if d.get("ktile"):
            rec["ktile_stamps_us_last_round"] = d["ktile"]
        if d.get("lat"):
            rec["lat_stamps_us_last_round"] = d["lat"]
        out[json.dumps(d["arm"])] = rec
        print(json.dumps(d["arm"]), json.dumps(rec), flush=True)
    print(json.dumps(out))
    for d in plans:
        d["plan"].close()


if __name__ == "__main__":
    main()
