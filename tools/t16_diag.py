"""Where the fp16 tile kernel's time goes (conv3x3_f16_tile_kernel, conv2-conv4 of the fp16 plan;
diagnostic build: FILE=kernels_f16.hip tools/build_diag.sh t16:-DT16DIAG=1, then
DNN_HIP_LIB=diag/libdnn_hip_t16.so).  Runs the batch-64 fp16 plan for --preheat seconds, then
reads the last launch's per-workgroup stamps of each layer (gemm_f16_tile.h T16_STAMP) and prints
the median cycles per phase: prologue, per (tile, chunk) pair the MFMA loop, the wait at the
pair's barrier (its successor's patch DMA) and the epilogue, and the launch span."""
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

WGS = 1024


def med(v):
    v = sorted(v)
    return "%7.0f (p10 %6.0f p90 %6.0f)" % (statistics.median(v), v[len(v) // 10], v[len(v) * 9 // 10])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preheat", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(a.batch, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    wb, sb = dnn_hip.Plan.memory(a.batch, (416, 416, 3), entries, precision="fp16")
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(sb, dtype=torch.uint8, device=dev)
    plan = dnn_hip.Plan(a.batch, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                        workspace_ptr=sbuf.data_ptr(), precision="fp16")
    print(plan.describe())
    x = torch.rand((a.batch, 416, 416, 3), device=dev)
    y = torch.empty((a.batch,) + tuple(plan.out_shape), device=dev)
    s = torch.cuda.Stream()
    t0 = time.time()
    while time.time() - t0 < a.preheat:
        for _ in range(10):
            plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
        s.synchronize()
    plan.timing_begin(3)
    for _ in range(3):
        plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
    ms, cnt = plan.timing_end()
    for k, m, c in zip(plan.kernels(), ms, cnt):
        print("  %-14s %.4f ms" % (k["name"], m / max(c, 1)))
    f = plan.lib.dnn_t16_diag_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    for k, name in enumerate(("conv2 (C 32)", "conv3 (C 64)", "conv4 (C 128)", "conv5 + pool5 (C 256)")):
        buf = (ctypes.c_ulonglong * (WGS * 32))()
        assert f(buf, k, WGS) == 0
        rows = [list(buf[32 * w:32 * w + 32]) for w in range(WGS) if buf[32 * w + 27] > 0]
        if not rows:
            print(name, ": no stamps")
            continue
        nch = {0: 1, 1: 2, 2: 4, 3: 8}[k]
        print("%s: %d workgroups, tiles/workgroup %s" % (name, len(rows), sorted(set(r[31] for r in rows))))
        print("  prologue              ", med([r[2] - r[1] for r in rows]))
        for q in range(8):
            mf, bw, ep = [], [], []
            for r in rows:
                if q >= r[31] * nch:
                    continue
                prev = r[2] if q == 0 else (r[3 + 3 * (q - 1) + 2] if (q - 1) % nch == nch - 1 else r[4 + 3 * (q - 1)])
                mf.append(r[3 + 3 * q] - prev)
                bw.append(r[4 + 3 * q] - r[3 + 3 * q])
                if q % nch == nch - 1:
                    ep.append(r[5 + 3 * q] - r[4 + 3 * q])
            if mf:
                print("  pair %d MFMA loop       %s" % (q, med(mf)))
                print("  pair %d barrier wait    %s" % (q, med(bw)))
                if ep:
                    print("  pair %d epilogue        %s" % (q, med(ep)))
        print("  total                 ", med([r[27] - r[1] for r in rows]))
        t0 = min(r[0] for r in rows)
        span = (max(r[28] for r in rows) - t0) * 10e-3
        clk = statistics.median([(r[27] - r[1]) / max(r[28] - r[0], 1) for r in rows]) * 100
        print("  span %.1f us, clock ~%.0f MHz" % (span, clk))


if __name__ == "__main__":
    main()
