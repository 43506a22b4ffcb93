"""Which streams share a hardware queue?  Two streams on one HW queue serialise even when
HIP has no dependency between them (GPU_MAX_HW_QUEUES=4 on the box).  For each pair (a, b):
a long spin kernel on a, then a short one on b; b finishing first means separate queues.
  python tools/stream_queue_probe.py [--nccl]   (--nccl: run under torch.distributed.run)"""
import os
import sys
import time

import torch


def overlaps(a, b, spin=200_000_000):
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    with torch.cuda.stream(a):
        torch.cuda._sleep(spin)
        ea.record(a)
    with torch.cuda.stream(b):
        torch.cuda._sleep(1000)
        eb.record(b)
    t0 = time.perf_counter()
    while not eb.query():
        if time.perf_counter() - t0 > 5:
            break
    first = eb.query() and not ea.query()
    torch.cuda.synchronize()
    return bool(first)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if "--nccl" in sys.argv:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)
        t = torch.ones(4, device=dev)
        tdist.all_reduce(t)
    streams = {"null": torch.cuda.default_stream(dev)}
    for i in range(4):
        streams[f"pool{i}"] = torch.cuda.Stream(dev)
    for i in range(3):
        streams[f"hi{i}"] = torch.cuda.Stream(dev, priority=-1)
    names = list(streams)
    print("queue-sharing matrix (X = serialised):", flush=True)
    for a in names:
        row = []
        for b in names:
            row.append("." if a == b else ("-" if overlaps(streams[a], streams[b]) else "X"))
        print(f"{a:>6} " + " ".join(row), flush=True)
    print("       " + " ".join(n[0] for n in names))
    print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))


if __name__ == "__main__":
    main()
