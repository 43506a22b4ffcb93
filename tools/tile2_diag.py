"""Where conv2 / conv3's time goes (conv3x3_x3_tile2_kernel, X3DIAG bit 1024 builds:
tools/build_diag.sh 1024, DNN_HIP_LIB=diag/libdnn_hip_d1024.so).  Runs the batch-64 fp32 plan back
to back for --preheat seconds, then reads the last launch's per-workgroup stamps of each layer
(gemm_x3_patch.h T2_DIAG_SLOTS) and prints the median cycles per phase, the launch span, and per
CU: workgroups, busy fraction (union of its workgroups' [start, end] over the span) and mean
concurrency (sum of durations over its busy time)."""
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

WGS, SLOTS = 4096, 16


def layer_report(name, rows):
    if not rows:
        print(name, ": no stamps")
        return
    print("%s: %d workgroups (wave 0, median cycles)" % (name, len(rows)))
    for nm, a, b in (("prologue (patch landed)", 1, 2), ("MFMA loop", 2, 3), ("epilogue + stores", 3, 4),
                     ("  fold + first barrier", 3, 12), ("  row table + barrier", 12, 13),
                     ("  pool/epilogue -> stage", 13, 14), ("  split-plane stores", 14, 4), ("total", 1, 4)):
        v = [r[b] - r[a] for r in rows]
        print("  %-24s %8.0f  (p10 %6.0f, p90 %6.0f)" % (nm, statistics.median(v), sorted(v)[len(v) // 10],
                                                          sorted(v)[len(v) * 9 // 10]))
    sk = [max(r[8:12]) - min(r[8:12]) for r in rows]
    print("  MFMA-end skew over the 4 waves  median %.0f (p90 %.0f)" % (statistics.median(sk), sorted(sk)[len(sk) * 9 // 10]))
    t0 = min(r[0] for r in rows)
    t1 = max(r[5] for r in rows)
    span = (t1 - t0) * 10e-3  # s_memrealtime: 100 MHz -> us
    cyc = statistics.median([(r[4] - r[1]) / max(r[5] - r[0], 1) for r in rows]) * 100  # MHz
    last_start = max(r[0] for r in rows)
    print("  launch span %.1f us (stamped), clock ~%.0f MHz, last workgroup starts at %.1f us" %
          (span, cyc, (last_start - t0) * 10e-3))
    cus = {}
    for r in rows:
        hw, xcc = r[6], r[7] & 0xf
        key = (xcc, (hw >> 8) & 0xff)
        cus.setdefault(key, []).append((r[0], r[5]))
    busy, conc, nwg = [], [], []
    for iv in cus.values():
        iv.sort()
        u, cs, ce = 0, None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    u += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        u += ce - cs
        busy.append(u / max(t1 - t0, 1))
        conc.append(sum(e - s for s, e in iv) / max(u, 1))
        nwg.append(len(iv))
    print("  CUs %d: workgroups/CU median %d (min %d, max %d); busy %.2f (min %.2f); concurrency %.2f" %
          (len(cus), statistics.median(nwg), min(nwg), max(nwg), statistics.median(busy), min(busy),
           statistics.median(conc)))
    # start-time histogram in tenths of the span
    h = [0] * 10
    for r in rows:
        h[min(9, int(10 * (r[0] - t0) / max(t1 - t0, 1)))] += 1
    print("  starts per tenth of span:", h)


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
    while time.time() - t0 < a.preheat:
        for _ in range(10):
            plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
        n += 10
        s.synchronize()
    plan.timing_begin(3)
    for _ in range(3):
        plan.run_device(a.batch, x.data_ptr(), y.data_ptr(), s.cuda_stream)
    ms, cnt = plan.timing_end()
    print("forwards %d" % n)
    for k, m, c in zip(plan.kernels(), ms, cnt):
        print("  %-14s %.4f ms" % (k["name"], m / max(c, 1)))
    fp = getattr(plan.lib, "dnn_pp_diag_stamps", None)
    if fp is not None:  # X3DIAG 2048: the ping-pong kernel's step cycles (conv2)
        fp.restype = ctypes.c_int
        fp.argtypes = [ctypes.c_void_p, ctypes.c_int]
        pb = (ctypes.c_ulonglong * (256 * 8))()
        assert fp(pb, 256) == 0
        rows = [list(pb[8 * w:8 * w + 8]) for w in range(256) if pb[8 * w + 6] > 0]
        print("ping-pong conv2: %d workgroups, median cycles per workgroup" % len(rows))
        for nm, i in (("team A MFMA steps", 0), ("team A store steps", 1), ("team A barrier waits", 2),
                      ("team B MFMA steps", 3), ("team B store steps", 4), ("team B barrier waits", 5),
                      ("total (wave 0)", 6)):
            print("  %-22s %10.0f" % (nm, statistics.median(r[i] for r in rows)))
    fc = getattr(plan.lib, "dnn_c16pp_diag_stamps", None)
    if fc is not None:  # X3DIAG 32768: conv1's ping-pong kernel's step cycles
        fc.restype = ctypes.c_int
        fc.argtypes = [ctypes.c_void_p, ctypes.c_int]
        cb = (ctypes.c_ulonglong * (512 * 16))()
        assert fc(cb, 512) == 0
        rows = [list(cb[16 * w:16 * w + 16]) for w in range(512) if cb[16 * w + 8] > 0]
        print("ping-pong conv1: %d workgroups, median cycles per workgroup (tiles of team A %d)" %
              (len(rows), statistics.median(r[9] for r in rows) if rows else 0))
        for nm, i in (("team A MFMA steps", 0), ("team A wait+split+loads", 1), ("team A epilogue+stores", 2),
                      ("team A barrier waits", 3), ("team B MFMA steps", 4), ("team B wait+split+loads", 5),
                      ("team B epilogue+stores", 6), ("team B barrier waits", 7), ("total (wave 0)", 8)):
            print("  %-24s %10.0f" % (nm, statistics.median(r[i] for r in rows)))
    fi = getattr(plan.lib, "dnn_img_diag_stamps", None)
    if fi is not None:  # X3DIAG 16384: the whole-image kernel's phases (conv5 + pool5)
        fi.restype = ctypes.c_int
        fi.argtypes = [ctypes.c_void_p, ctypes.c_int]
        ib = (ctypes.c_ulonglong * (512 * 8))()
        assert fi(ib, 512) == 0
        rows = [list(ib[8 * w:8 * w + 8]) for w in range(512) if ib[8 * w + 7] > 0]
        print("conv5 + pool5 (whole-image tiles): %d workgroups, median cycles" % len(rows))
        for nm, a, b in (("prologue", 1, 2), ("loop (wave 0)", 2, 3), ("loop (wave 7)", 2, 4),
                         ("fold + stage", 3, 5), ("pool/epilogue/stores", 5, 6), ("total", 1, 6)):
            v = sorted(r[b] - r[a] for r in rows)
            print("  %-24s %8.0f  (p10 %6.0f, p90 %6.0f)" % (nm, statistics.median(v), v[len(v) // 10], v[len(v) * 9 // 10]))
        t0 = min(r[0] for r in rows)
        print("  span %.1f us" % ((max(r[7] for r in rows) - t0) * 10e-3))
    fa = getattr(plan.lib, "dnn_acc2_diag_stamps", None)
    if fa is not None:  # X3DIAG 8192: the wide kernel's phases per layer class
        fa.restype = ctypes.c_int
        fa.argtypes = [ctypes.c_void_p, ctypes.c_int]
        ab = (ctypes.c_ulonglong * (3 * 512 * 8))()
        assert fa(ab, 3 * 512) == 0
        for li, name in enumerate(("conv4 (N = 256)", "conv5 (N = 512)", "conv6/7 (N = 1024, last)")):
            rows = [list(ab[(li * 512 + w) * 8:(li * 512 + w) * 8 + 8]) for w in range(512)]
            rows = [r for r in rows if r[5] > 0 and r[4] > 0]
            if not rows:
                continue
            print("%s: %d workgroups, median cycles" % (name, len(rows)))
            for nm, a, b in (("prologue", 1, 2), ("main loop", 2, 3), ("epilogue", 3, 4), ("total", 1, 4)):
                v = sorted(r[b] - r[a] for r in rows)
                print("  %-10s %8.0f  (p10 %6.0f, p90 %6.0f)" % (nm, statistics.median(v), v[len(v) // 10], v[len(v) * 9 // 10]))
            t0 = min(r[0] for r in rows)
            t1 = max(r[5] for r in rows)
            st = sorted((r[0] - t0) * 10e-3 for r in rows)
            en = sorted((r[5] - t0) * 10e-3 for r in rows)
            cyc = statistics.median([(r[4] - r[1]) / max(r[5] - r[0], 1) for r in rows]) * 100
            print("  span %.1f us, clock ~%.0f MHz; starts p50 %.1f max %.1f us; ends p10 %.1f p50 %.1f max %.1f us" %
                  ((t1 - t0) * 10e-3, cyc, st[len(st) // 2], st[-1], en[len(en) // 10], en[len(en) // 2], en[-1]))
    fn = getattr(plan.lib, "dnn_tile2_diag_stamps", None)
    if fn is None:
        print("no dnn_tile2_diag_stamps: not an X3DIAG 1024 build")
        return
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nw = 2 * WGS * SLOTS
    buf = (ctypes.c_ulonglong * nw)()
    assert fn(buf, nw) == 0
    for li, name in enumerate(("conv2 (N = 64)", "conv3 (N = 128)")):
        rows = []
        for wg in range(WGS):
            v = list(buf[(li * WGS + wg) * SLOTS:(li * WGS + wg + 1) * SLOTS])
            if v[5] > 0 and v[4] > 0:
                rows.append(v)
        layer_report(name, rows)


if __name__ == "__main__":
    main()
