"""In-process A/B of launch-time switches on the batch-64 fp32 plan (cdna_hip_programming.md
§5.4 rule 24: variants interleaved in one process, after a >= 2 s pre-heat at the clock the
chip holds under load).

  python tools/x3_ab.py --env DNN_HIP_X3_C16P=0,2 [--env DNN_AB_DUMMY=a,b] [--rounds 6] [--iters 20] [--preheat 3]

Only switches read per launch take effect between arms (DNN_HIP_X3_C16P; a switch no code reads, e.g. DNN_AB_DUMMY, gives null arms: the noise floor).  Prints, per arm, the
median over rounds of each kernel's mean HIP-event time and of the forward.  With a library
built with X3DIAG bit 16 (tools/build_diag.sh 16, DNN_HIP_LIB=diag/libdnn_hip_d16.so) it also
reads the wide x3 kernel's per-workgroup s_memtime / s_memrealtime stamps of the last conv7
launch: the in-kernel clock (MI355X_MICROARCH, DVFS give-back item 6)."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dnn-inference-engine_amd"))

import torch  # noqa: E402

import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402


def clock_stamps(lib, nwg):
    fn = getattr(lib, "dnn_x3_diag_stamps", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (4 * nwg))()
    if fn(buf, nwg) != 0:
        return None
    ghz, loop_us, cyc, rows = [], [], [], []
    for w in range(nwg):
        t0, r0, t1, r1 = buf[4 * w:4 * w + 4]
        if r1 > r0 and t1 > t0:
            ghz.append((t1 - t0) / (r1 - r0) * 0.1)  # s_memrealtime ticks at 100 MHz
            loop_us.append((r1 - r0) / 100.0)
            cyc.append(t1 - t0)
            rows.append((w, r0, r1, t1 - t0))
    if not ghz:
        return None
    r0min = min(r[1] for r in rows)
    # per XCD (blocks b and b + 8 share one: b % 8): clock, loop time, loop start and end
    # relative to the earliest loop start (us)
    xcd = {}
    for x in range(8):
        sel = [r for r in rows if r[0] % 8 == x]
        if not sel:
            continue
        xcd[x] = {"ghz": round(statistics.median(r[3] / (r[2] - r[1]) * 0.1 for r in sel), 4),
                  "loop_us": round(statistics.median((r[2] - r[1]) / 100 for r in sel), 2),
                  "start_us_max": round(max((r[1] - r0min) / 100 for r in sel), 2),
                  "end_us_max": round(max((r[2] - r0min) / 100 for r in sel), 2),
                  "mcycles": round(statistics.median(r[3] for r in sel) / 1e6, 4)}
    return {"median_ghz": round(statistics.median(ghz), 4), "min_ghz": round(min(ghz), 4),
            "max_ghz": round(max(ghz), 4), "median_loop_us": round(statistics.median(loop_us), 2),
            "max_loop_us": round(max(loop_us), 2), "workgroups": len(ghz),
            "mcycles_median": round(statistics.median(cyc) / 1e6, 4), "mcycles_min": round(min(cyc) / 1e6, 4),
            "mcycles_max": round(max(cyc) / 1e6, 4),
            "span_us": round((max(r[2] for r in rows) - r0min) / 100, 2), "per_xcd": xcd}


C16_SLOTS = ["drain", "split", "bar1", "mfma", "bar2", "epi_math", "stores", "bar3"]


def c16_phases(lib, nwg=512):
    """X3DIAG bit 32 builds: conv1's persistent x3 kernel, wave 0's s_memtime sums per phase
    (c16_diag_stamps, last launch); medians over workgroups of cycles per tile."""
    fn = getattr(lib, "dnn_c16_diag_stamps", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ns = 10
    buf = (ctypes.c_ulonglong * (ns * nwg))()
    if fn(buf, nwg) != 0:
        return None
    rows = [buf[ns * w:ns * w + ns] for w in range(nwg) if buf[ns * w + 8] > 0]
    if not rows:
        return None
    out = {"workgroups": len(rows), "tiles_median": statistics.median(r[8] for r in rows)}
    for k, name in enumerate(C16_SLOTS):
        out[name] = round(statistics.median(r[k] / r[8] for r in rows))
    tot = [sum(r[:8]) for r in rows]
    out["total_mcycles_median"] = round(statistics.median(tot) / 1e6, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", action="append", default=[], help="VAR=v1,v2,... (arms)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--preheat", type=float, default=3.0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--kernels", default="conv0,conv1,conv2,conv3,conv4,conv5,conv6,conv7,conv8")
    a = ap.parse_args()
    arms = [{}]
    for spec in a.env:
        var, vals = spec.split("=", 1)
        arms = [dict(x, **{var: v}) for x in arms for v in vals.split(",")]
    dev = torch.device("cuda", 0)
    B = a.batch
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(B, 416, 416, 3))
    plan = dnn_hip.Plan.from_graph(g, device=0, precision=a.precision)
    frames = torch.rand((B, 416, 416, 3), generator=torch.Generator(device=dev).manual_seed(7), device=dev)
    out = torch.empty((B,) + plan.out_shape, device=dev)
    stream = torch.cuda.Stream(dev)
    sp = stream.cuda_stream
    names = [k["name"] for k in plan.kernels()]
    base = dict(os.environ)

    def set_arm(arm):
        for k in {k for x in arms for k in x}:
            if k in base:
                os.environ[k] = base[k]
            else:
                os.environ.pop(k, None)
        os.environ.update(arm)

    def fwd(n):
        for _ in range(n):
            plan.run_device(B, frames.data_ptr(), out.data_ptr(), sp)

    t0 = time.time()
    set_arm(arms[0])
    fwd(3)
    stream.synchronize()
    cold = clock_stamps(plan.lib, 4096)
    while time.time() - t0 < a.preheat:
        fwd(20)
        stream.synchronize()
    res = {json.dumps(x): {"fwd_ms": [], "k": {n: [] for n in names}, "clock": []} for x in arms}
    for r in range(a.rounds):
        # arm order rotated and reversed round by round (no arm always follows the same one:
        # the clock a kernel runs at depends on the power drawn just before it)
        order = arms[r % len(arms):] + arms[:r % len(arms)]
        if r % 2:
            order = order[::-1]
        for arm in order:
            set_arm(arm)
            fwd(2)
            plan.timing_begin(a.iters)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fwd(a.iters)
            e1.record(stream)
            stream.synchronize()
            ms, cnt = plan.timing_end()
            d = res[json.dumps(arm)]
            d["fwd_ms"].append(e0.elapsed_time(e1) / a.iters)
            for i, n in enumerate(names):
                d["k"][n].append(ms[i] / max(cnt[i], 1))
            c = clock_stamps(plan.lib, 4096)
            if c:
                d["clock"].append(c)
            c = c16_phases(plan.lib)
            if c:
                d.setdefault("c16", []).append(c)
    want = [n for n in names if n.split(".")[0] in a.kernels.split(",")]
    summary = {"cold_clock": cold, "arms": {}}
    for key, d in res.items():
        s = {"fwd_ms_median": round(statistics.median(d["fwd_ms"]), 4), "fwd_ms_min": round(min(d["fwd_ms"]), 4),
             "kernels_ms_median": {n: round(statistics.median(d["k"][n]), 4) for n in want},
             "kernels_ms_min": {n: round(min(d["k"][n]), 4) for n in want}}
        if d.get("c16"):
            s["c16_phases_last_round"] = d["c16"][-1]
        if d["clock"]:
            s["clock_last_round"] = d["clock"][-1]
            s["clock_median_ghz_over_rounds"] = round(statistics.median(c["median_ghz"] for c in d["clock"]), 4)
        summary["arms"][key] = s
        print(key, json.dumps(s), flush=True)
    print(json.dumps(summary))
    plan.close()


if __name__ == "__main__":
    main()
