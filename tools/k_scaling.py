"""K-scaling probe for the fp32 implicit GEMM: one 3x3 SAME conv + BN + leaky + 2x2/s2 pool at
conv3's M and N (batch 64, 52x52, 128 outputs) with the input channels swept, so K = 9*C
grows with M, N and the tile grid fixed.  TFLOP/s that rises with K means per-tile fixed cost
(address setup, the first stage's DMA latency, the epilogue) is what holds the short-K layers
back.  Run on a GPU box: python tools/k_scaling.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dnn-inference-engine_amd"))
import dnn_hip  # noqa: E402


def layer(B, H, W, C, OC, steps=20):
    rng = np.random.default_rng(0)
    g = dnn_hip.DnnGraphBuilder()
    y = g.create_input([B, H, W, C])
    y = g.create_conv2d(y, (rng.standard_normal((3, 3, C, OC)) * 0.05).astype(np.float32), [1, 1, 1, 1], "SAME")
    y = g.create_batch_norm(y, np.zeros(OC, np.float32), np.ones(OC, np.float32), np.ones(OC, np.float32), 1e-5)
    y = g.create_leaky_relu(y)
    y = g.create_max_pool2d(y, [1, 2, 2, 1], [1, 2, 2, 1], "SAME")
    g.set_out_node(y)
    entries = dnn_hip.lower_graph(g)
    dev = torch.device("cuda", 0)
    wb, sb = dnn_hip.Plan.memory(B, (H, W, C), entries)
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
    p = dnn_hip.Plan(B, (H, W, C), entries, device=0, weights_ptr=wbuf.data_ptr(), workspace_ptr=sbuf.data_ptr())
    x = torch.rand((B, H, W, C), device=dev)
    out = torch.empty((B, (H + 1) // 2, (W + 1) // 2, OC), device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        p.run_device(B, x.data_ptr(), out.data_ptr(), s)
    torch.cuda.synchronize()
    p.timing_begin(steps)
    for _ in range(steps):
        p.run_device(B, x.data_ptr(), out.data_ptr(), s)
    ms, cnt = p.timing_end()
    k = p.kernels()[0]
    avg = ms[0] / max(cnt[0], 1)
    desc = p.describe().splitlines()[-1] if hasattr(p, "describe") else ""
    p.close()
    return avg, k["flops"] / (avg / 1e3) / 1e12, desc


def main():
    for C in (32, 64, 128, 256):
        ms, tf, desc = layer(64, 52, 52, C, 128)
        print(f"C={C:4d} K={9 * C:5d}  {ms:8.4f} ms  {tf:7.1f} TF   {desc}", flush=True)
    for C in (64, 128, 256, 512):
        ms, tf, desc = layer(64, 104, 104, C, 64)
        print(f"N=64 104x104 C={C:4d} K={9 * C:5d}  {ms:8.4f} ms  {tf:7.1f} TF   {desc}", flush=True)


if __name__ == "__main__":
    main()
