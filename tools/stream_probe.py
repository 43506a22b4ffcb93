"""Multi-stream probe: does running a 64-frame batch as S sub-batches on S HIP streams (one
plan + workspace per stream, one shared weight arena) beat one 64-frame forward?  Each layer's
last workgroup round leaves CUs idle (tile quantization: conv4 has 676 128x128 tiles for 512
slots); concurrent sub-batches can fill those tails with the other stream's layers.

  python tools/stream_probe.py [--steps 30]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dnn-inference-engine_amd"))
import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    ws = synth.yolo_weights()
    frames = torch.rand((B, 416, 416, 3), device=dev)
    out = torch.empty((B, 13, 13, 125), device=dev)
    wbuf = None
    results = {}
    ref = None
    for S in (1, 2, 4):
        b = B // S
        g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(b, 416, 416, 3))
        entries = dnn_hip.lower_graph(g)
        wb, sb = dnn_hip.Plan.memory(b, (416, 416, 3), entries, precision=a.precision)
        if wbuf is None:
            wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
        plans, bufs = [], []
        for s in range(S):
            sbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
            bufs.append(sbuf)
            plans.append(dnn_hip.Plan(b, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                                      workspace_ptr=sbuf.data_ptr(), upload=True, precision=a.precision))
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        main_s = torch.cuda.current_stream(dev)

        def step():
            ev = torch.cuda.Event()
            ev.record(main_s)
            for s in range(S):
                streams[s].wait_event(ev)
                plans[s].run_device(b, frames[s * b:].data_ptr(), out[s * b:].data_ptr(), streams[s].cuda_stream)
            for s in range(S):
                e = torch.cuda.Event()
                e.record(streams[s])
                main_s.wait_event(e)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(main_s)
        for _ in range(a.steps):
            step()
        t1.record(main_s)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.steps
        if ref is None:
            ref = out.clone()
        same = bool(torch.equal(out, ref))
        results[S] = ms
        print(f"S={S} sub-batch {b}: {ms:.3f} ms per {B} frames = {B / ms * 1e3:.0f} img/s, identical={same}",
              flush=True)
        del plans, bufs


if __name__ == "__main__":
    main()
