"""Where the fused front kernel's time goes (conv_front.hip, FRONTDIAG builds: tools/build_diag.sh
with FILE=conv_front.hip "fd1:-DFRONTDIAG=1", DNN_HIP_LIB=diag/libdnn_hip_fd1.so).  Runs the
batch-64 fp32 plan back to back for --preheat seconds on random frames, then reads the per-wave
s_memtime sums of the last front launch and prints, per role, the median over workgroups of the
cycles per tile in each phase (slots: conv_front.hip FRONTDIAG)."""
import argparse
import ctypes
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

SLOTS = 6
NAMES = {"producer": ["total", "wait_free", "conv0", "-", "frame_meet", "tiles"],
         "consumer": ["total", "wait_full", "-", "conv1", "-", "tiles"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preheat", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(a.batch, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    wb, sb = dnn_hip.Plan.memory(a.batch, (416, 416, 3), entries)
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(sb, dtype=torch.uint8, device=dev)
    plan = dnn_hip.Plan(a.batch, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                        workspace_ptr=sbuf.data_ptr())
    x = torch.rand((a.batch, 416, 416, 3), device=dev)
    y = torch.empty((a.batch, 13, 13, 125), device=dev)
    s = torch.cuda.Stream()
    t0 = time.time()
    n = 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    while time.time() - t0 < a.preheat:
        for _ in range(10):
            plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
        n += 10
        s.synchronize()
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(10):
            plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
        e1.record(s)
    s.synchronize()
    print("forwards %d, %.4f ms per forward" % (n, e0.elapsed_time(e1) / 10))
    plan.timing_begin(3)
    for _ in range(3):
        plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
    ms, cnt = plan.timing_end()
    for k, m, c in zip(plan.kernels(), ms, cnt):
        print("  %-14s %.4f ms" % (k["name"], m / max(c, 1)))
    lib = plan.lib
    fn = getattr(lib, "dnn_front_diag_stamps", None)
    if fn is None:
        print("no dnn_front_diag_stamps: not a FRONTDIAG build")
        return
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nw = 256 * 16 * SLOTS
    buf = (ctypes.c_ulonglong * nw)()
    got = fn(buf, nw)
    assert got > 0, got
    for role, waves in (("producer", range(8)), ("consumer", range(8, 16))):
        rows = []
        for wg in range(256):
            for w in waves:
                v = buf[(wg * 16 + w) * SLOTS:(wg * 16 + w + 1) * SLOTS]
                if v[5] > 0:
                    rows.append([v[i] / v[5] for i in range(5)] + [v[5]])
        if not rows:
            continue
        print(role, "(median over %d waves, cycles per tile)" % len(rows))
        for i, nm in enumerate(NAMES[role]):
            if nm != "-":
                print("  %-12s %10.0f" % (nm, statistics.median(r[i] for r in rows)))


if __name__ == "__main__":
    main()
