"""Data-parallel sharding of a frame batch across the GPUs of one node.

The reference is single-process and single-device; the multi-GPU layer is new.  Frames
are independent, so a global batch is split into contiguous per-rank shards with no
exchange between layers.  The only collectives are the two the north star names:
  * one broadcast of the packed weight buffer from rank 0 at start-up (63.5 MB fp32);
  * one gather of the per-rank outputs to rank 0 per batch ([n,13,13,125] fp32 per rank).
One process per GPU, torch.distributed over RCCL ("nccl" backend) on the GPU box, gloo
for the CPU tests; the compute step is injected, so the same runner drives the HIP plan
(bench.py) and a CPU stand-in (tests/test_dist_cpu.py).
"""
import os

import torch
import torch.distributed as dist


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


def broadcast_weights(buf, src=0):
    """Broadcast a flat weight tensor in place from `src` (once, at start-up)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(buf, src=src)
    return buf


def gather_outputs(local, dst=0):
    """Gather equal-shaped per-rank output tensors to `dst`; returns the concatenation on
    `dst` (rank order = shard order) and None elsewhere.  Shards of unequal size are padded
    to the largest by the caller (see ShardedRunner)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    parts = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    dist.gather(local, parts, dst=dst)
    return torch.cat(parts, 0) if rank == dst else None


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
