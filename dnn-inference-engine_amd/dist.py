"""Data-parallel sharding of a frame batch across the GPUs of one node.

The reference is single-process and single-device; the multi-GPU layer is new.  Frames
are independent, so a global batch is split into contiguous per-rank shards with no
exchange between layers.  The only collectives are the ones the north star names:
  * one broadcast of the packed weight buffer from rank 0 at start-up (63.5 MB fp32);
  * per batch, a gather to rank 0 of either the raw outputs ([n,13,13,125] fp32 per rank,
    gather_outputs) or — after the on-GPU postprocessing (yolo_post.py) — only the packed
    detections (40 B each, gather_detections: a few kB per image instead of 84.5 kB).
One process per GPU, torch.distributed over RCCL ("nccl" backend) on the GPU box, gloo
for the CPU tests; the compute step is injected, so the same runner drives the HIP plan
(bench.py) and a CPU stand-in (tests/test_dist_cpu.py).
"""
import os

import numpy as np
import torch
import torch.distributed as dist

# dnn_detection of include/dnn_hip_post.h (= yolo_post.DETECTION_DTYPE; kept here so the
# gather needs no HIP library)
DETECTION_DTYPE = np.dtype([("cls", "<i4"), ("score", "<f4"), ("left", "<i8"), ("top", "<i8"), ("right", "<i8"),
                            ("bottom", "<i8")])


def shard_range(total, world, rank):
    """Contiguous balanced shard [start, start+count) of `total` frames for `rank`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} for world {world}")
    base, extra = divmod(int(total), int(world))
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def env_rank():
    """(rank, local_rank, world_size) from torch.distributed.run's environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend, device=None):
    """Initialise the default process group once (127.0.0.1 rendezvous from the env)."""
    if dist.is_available() and not dist.is_initialized():
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = device
        dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size()


def _host_staged(t):
    """gloo runs collectives on host memory: with device tensors (the one-GPU multi-rank
    rehearsal, DNN_BENCH_BACKEND=gloo) each collective goes through a CPU copy.  RCCL
    ("nccl") works on the device tensors directly."""
    return t.is_cuda and dist.get_backend() == "gloo"


def broadcast_weights(buf, src=0):
    """Broadcast a flat weight tensor in place from `src` (once, at start-up)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        if _host_staged(buf):
            h = buf.cpu()
            dist.broadcast(h, src=src)
            buf.copy_(h)
        else:
            dist.broadcast(buf, src=src)
    return buf


def _gather(t, parts, dst):
    if _host_staged(t):
        hp = [torch.empty(p.shape, dtype=p.dtype) for p in parts] if parts is not None else None
        dist.gather(t.cpu(), hp, dst=dst)
        if parts is not None:
            for p, h in zip(parts, hp):
                p.copy_(h)
    else:
        dist.gather(t, parts, dst=dst)


def _all_gather(parts, t):
    if _host_staged(t):
        hp = [torch.empty(p.shape, dtype=p.dtype) for p in parts]
        dist.all_gather(hp, t.cpu())
        for p, h in zip(parts, hp):
            p.copy_(h)
    else:
        dist.all_gather(parts, t)


def gather_outputs(local, dst=0):
    """Gather equal-shaped per-rank output tensors to `dst`; returns the concatenation on
    `dst` (rank order = shard order) and None elsewhere.  Shards of unequal size are padded
    to the largest by the caller (see ShardedRunner)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    parts = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    _gather(local, parts, dst)
    return torch.cat(parts, 0) if rank == dst else None


def gather_detections(packed, total, counts, n, dst=0):
    """Gather this rank's packed detections to `dst`.

    packed  [rows, 40] uint8 tensor: the rank's detections image-major (yolo_post
            DetectionBuffers.pack / dnn_yolo_pack_detections), rows >= total
    total   [1] int32 tensor: valid rows of `packed`
    counts  [cap] int32 tensor: detections per image (< 0: the image's error code)
    n       valid images of this rank's shard
    Returns on `dst` (dets_u8 [P, 40] numpy, counts [sum of n over ranks] numpy int32) in
    global (rank, image) order; None elsewhere.  One scalar sync for the row count, then
    (N > 1) an all_gather of two scalars and gathers of max_rank(P) * 40 B and the counts."""
    p = int(total.item())
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return packed[:p].cpu().numpy(), counts[:n].cpu().numpy()
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = packed.device
    sizes = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    _all_gather(sizes, torch.tensor([p, n], dtype=torch.int64, device=dev))
    sizes = [tuple(int(v) for v in t.cpu()) for t in sizes]
    pmax, nmax = max(max(sz[0] for sz in sizes), 1), max(max(sz[1] for sz in sizes), 1)
    if packed.shape[0] >= pmax:
        pbuf = packed[:pmax].contiguous()
    else:
        pbuf = torch.zeros((pmax, packed.shape[1]), dtype=torch.uint8, device=dev)
        pbuf[:p] = packed[:p]
    cbuf = torch.zeros(nmax, dtype=torch.int32, device=dev)
    cbuf[:n] = counts[:n]
    pparts = [torch.empty_like(pbuf) for _ in range(world)] if rank == dst else None
    cparts = [torch.empty_like(cbuf) for _ in range(world)] if rank == dst else None
    _gather(pbuf, pparts, dst)
    _gather(cbuf, cparts, dst)
    if rank != dst:
        return None
    d = torch.cat([pparts[r][:sizes[r][0]] for r in range(world)], 0).cpu().numpy()
    cnt = torch.cat([cparts[r][:sizes[r][1]] for r in range(world)], 0).cpu().numpy()
    return d, cnt


def unpack_detections(dets_u8, counts):
    """(packed [P, 40] uint8, counts) from gather_detections -> per image a list of
    (class, left, top, right, bottom, score), or the negative error code."""
    rows = np.ascontiguousarray(dets_u8).reshape(-1, 40).view(DETECTION_DTYPE).reshape(-1) if len(dets_u8) else []
    out, pos = [], 0
    for n in counts:
        n = int(n)
        if n < 0:
            out.append(n)
            continue
        out.append([(int(d["cls"]), int(d["left"]), int(d["top"]), int(d["right"]), int(d["bottom"]),
                     float(d["score"])) for d in rows[pos:pos + n]])
        pos += n
    return out


class ShardedRunner(object):
    """Runs `compute(inp, out, n)` on this rank's shard of a global batch and gathers.

    compute   callable writing outputs for the first n frames of `inp` into `out`
    in_shape  per-frame input shape, out_shape per-frame output shape
    """

    def __init__(self, compute, global_batch, in_shape, out_shape, device, dtype=torch.float32):
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.global_batch = int(global_batch)
        self.start, self.count = shard_range(self.global_batch, self.world, self.rank)
        self.shard_cap = -(-self.global_batch // self.world)  # ceil: equal-size gather buffers
        self.compute = compute
        self.out = torch.zeros((self.shard_cap,) + tuple(out_shape), dtype=dtype, device=device)
        self.in_shape = tuple(in_shape)

    def local_slice(self, global_frames):
        return global_frames[self.start:self.start + self.count]

    def step(self, local_in):
        """One batch: local compute, then gather to rank 0 (returns [global_batch, ...]
        on rank 0, None on other ranks)."""
        self.compute(local_in, self.out, self.count)
        full = gather_outputs(self.out)
        if full is None:
            return None
        if self.world == 1:
            return full[:self.count]
        # drop the per-rank padding rows
        rows = []
        for r in range(self.world):
            s, c = shard_range(self.global_batch, self.world, r)
            rows.append(full[r * self.shard_cap:r * self.shard_cap + c])
        return torch.cat(rows, 0)

    def launch_detections(self, local_in, post, slot):
        """Pipelined form of step_detections, first half: enqueue the forward for this rank's
        shard into output slot `slot` (0/1) on the current stream, and `post(out, n, slot,
        stream_ptr)` (postprocess + pack) on a post stream that waits only for that forward,
        without waiting; returns a handle for finish_detections.  The postprocessing of step
        k (one workgroup per image: a quarter of the CUs) thus runs beside step k+1's first
        layers instead of between the two forwards.  The slot's previous gather must have
        been finished (its reads are ordered before this launch, and through the forward's
        event before this post)."""
        dev = self.out.device
        if not hasattr(self, "_outs"):
            self._outs = [self.out, torch.zeros_like(self.out)]
            self._side = torch.cuda.Stream(dev)
            self._post = torch.cuda.Stream(dev)
            self._freed = [None, None]
        cur = torch.cuda.current_stream(dev)
        if self._freed[slot] is not None:
            cur.wait_event(self._freed[slot])
        out = self._outs[slot]
        self.compute(local_in, out, self.count)
        done = torch.cuda.Event()
        done.record(cur)
        self._post.wait_event(done)
        with torch.cuda.stream(self._post):
            packed, total, counts = post(out, self.count, slot, self._post.cuda_stream)
        ready = torch.cuda.Event()
        ready.record(self._post)
        return slot, packed, total, counts, ready

    def finish_detections(self, handle):
        """Second half: on a side stream that waits only for that step's pack (so later steps
        already enqueued keep the GPU busy), read the row count and gather the packed
        detections (as gather_detections).  Returns what step_detections returns."""
        slot, packed, total, counts, ready = handle
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            r = gather_detections(packed, total, counts, self.count)
            freed = torch.cuda.Event()
            freed.record(self._side)
        self._freed[slot] = freed
        return r

    def step_detections(self, local_in, post):
        """One batch ending in detections: local compute, then `post(out, n)` -> (packed
        [rows, 40] uint8, total [1] int32, counts [cap] int32) on this rank's device (the
        on-GPU postprocessing + pack), then the packed detection gather.  Returns (dets_u8
        [P, 40], counts [global_batch]) on rank 0 (unpack_detections turns them into rows),
        None elsewhere."""
        self.compute(local_in, self.out, self.count)
        packed, total, counts = post(self.out, self.count)
        return gather_detections(packed, total, counts, self.count)
