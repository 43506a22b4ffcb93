"""Data-parallel sharding of a frame batch across the GPUs of one node.

The reference is single-process and single-device; the multi-GPU layer is new.  Frames
are independent, so a global batch is split into contiguous per-rank shards with no
exchange between layers.  The only collectives are the ones the north star names:
  * one broadcast of the packed weight buffer from rank 0 at start-up (63.5 MB fp32);
  * per batch, a gather to rank 0 of either the raw outputs ([n,13,13,125] fp32 per rank,
    gather_outputs) or — after the on-GPU postprocessing (yolo_post.py) — the packed
    detections (DetectionGather: sizes all-gathered, then max-over-ranks valid rows; the
    "deferred" mode reads the sizes on the host one step after their all-gather, so no
    host ever waits on the step it is finishing; or a fixed-capacity buffer sent without
    any host synchronisation).
One process per GPU, torch.distributed over RCCL ("nccl" backend) on the GPU box, gloo
for the CPU tests; the compute step is injected, so the same runner drives the HIP plan
(bench.py) and a CPU stand-in (tests/test_dist_cpu.py).
"""
import os
import time
from contextlib import nullcontext as _nullcontext

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


def _collectives():
    """Collectives run whenever a process group exists — also at world size 1, so a
    one-process RCCL group executes the same broadcast/gather code the 8-GPU job does."""
    return dist.is_available() and dist.is_initialized()


def broadcast_weights(buf, src=0):
    """Broadcast a flat weight tensor in place from `src` (once, at start-up)."""
    if _collectives():
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


def gather_outputs(local, dst=0):
    """Gather equal-shaped per-rank output tensors to `dst`; returns the concatenation on
    `dst` (rank order = shard order) and None elsewhere.  Shards of unequal size are padded
    to the largest by the caller (see ShardedRunner)."""
    if not _collectives():
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    parts = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    _gather(local, parts, dst)
    return torch.cat(parts, 0) if rank == dst else None


class DetectionGather(object):
    """Gather of every rank's packed detections to `dst` (the "gather of
    detections").  Per step each rank contributes
      meta    int32 [2 + cap]: valid rows of `packed`, valid images n, counts[:cap]
              (counts < 0: that image's error code);
      payload rows of its packed buffer [cap * max_det, 40] uint8 (image-major).
    Two modes:
      "sized" (default)  meta is all-gathered (fixed size, 264 B at cap 64), every rank reads
              the sizes on the host and the payload gather moves max-over-ranks valid rows
              (≈45 detections per image with the synthetic weights: ≈115 kB per rank).  The
              host read waits for that step on all ranks, so the caller keeps steps in
              flight (ShardedRunner: three) and the wait is on a step whose successors are
              already queued on the GPU;
      "deferred"  as "sized", split in two: launch_meta() enqueues the meta all-gather and an
              asynchronous copy of it into pinned host memory; launch_payload(), called one
              step later, reads the sizes there (the copy has long completed unless some rank
              is more than a step behind) and enqueues the payload gather.  Every rank's host
              touches a step's sizes only after it has enqueued the next step's meta, so the
              cross-rank rendezvous of "sized" (each host waiting for that step on all ranks)
              moves one step further behind the GPU queue; the caller keeps one more output
              slot than steps in flight (ShardedRunner.inflight);
      "fixed"  meta is gathered to `dst` and the payload is the whole packed buffer (its
              capacity is the most detections `cap` images can have, 845 each: 2.16 MB per
              rank at 64 images), so no rank ever reads a size on the host before sending and
              non-root ranks never wait; costs a longer RCCL kernel per step beside the
              forward (measured: 0.13 ms at one rank vs 0.02 ms sized).
    Receive buffers are allocated once per slot."""

    MODES = ("sized", "deferred", "fixed")

    def __init__(self, cap, rows, device, slots=2, dst=0, mode="sized"):
        if mode not in self.MODES:
            raise ValueError(f"mode {mode!r}")
        self.cap, self.rows, self.dst, self.mode = int(cap), int(rows), dst, mode
        self.rank = dist.get_rank() if _collectives() else 0
        self.world = dist.get_world_size() if _collectives() else 1
        self.meta = [torch.zeros(2 + self.cap, dtype=torch.int32, device=device) for _ in range(slots)]
        root = self.rank == dst
        coll = _collectives()
        all_meta = coll and mode in ("sized", "deferred")
        self.mparts = [[torch.empty_like(m) for _ in range(self.world)] if coll and (root or all_meta) else None
                       for m in self.meta]
        self.pparts = [[torch.empty((self.rows, 40), dtype=torch.uint8, device=device) for _ in range(self.world)]
                       if coll and root else None for _ in range(slots)]
        # deferred: the all-gathered meta of each slot lands here (pinned: the copy is async)
        pin = torch.device(device).type == "cuda"
        self.hmeta = [torch.zeros((self.world, 2 + self.cap), dtype=torch.int32, pin_memory=pin)
                      if all_meta and mode == "deferred" else None for _ in range(slots)]

    def _stage_meta(self, slot, total, counts, n):
        meta = self.meta[slot]
        meta[0:1].copy_(total[:1], non_blocking=True)
        meta[1].fill_(int(n))
        k = min(self.cap, counts.shape[0])
        meta[2:2 + k].copy_(counts[:k], non_blocking=True)
        return meta

    def _all_gather_meta(self, slot, meta):
        mparts = self.mparts[slot]
        if _host_staged(meta):
            hp = [torch.empty(p.shape, dtype=p.dtype) for p in mparts]
            dist.all_gather(hp, meta.cpu())
            for p, h in zip(mparts, hp):
                p.copy_(h)
        else:
            dist.all_gather(mparts, meta)
        return mparts

    def _payload(self, slot, packed, sizes):
        """Enqueue the payload gather of max-over-ranks valid rows (sizes: numpy [world, ...])."""
        pmax = int(sizes[:, 0].max())
        pparts = self.pparts[slot]
        if pmax > 0:
            _gather(packed[:pmax], [p[:pmax] for p in pparts] if self.rank == self.dst else None, self.dst)
        return pparts

    def _handle(self, mparts, pparts, sizes, packed):
        done, stream = None, None
        if packed.is_cuda:
            stream = torch.cuda.current_stream(packed.device)
            done = torch.cuda.Event()
            done.record(stream)
        return (mparts, pparts, sizes) if self.rank == self.dst else None, done, stream

    def launch_meta(self, slot, packed, total, counts, n):
        """deferred, first half: enqueue slot `slot`'s meta all-gather and its asynchronous
        copy to pinned host memory on the current stream; nothing waits on the host.  Returns
        a handle for launch_payload()."""
        if self.mode != "deferred":
            raise ValueError("launch_meta is the deferred mode's first half")
        if packed.shape[0] != self.rows:
            raise ValueError(f"packed has {packed.shape[0]} rows, the gather was sized for {self.rows}")
        meta = self._stage_meta(slot, total, counts, n)
        if not _collectives():
            return slot, packed, [meta], None
        mparts = self._all_gather_meta(slot, meta)
        hm = self.hmeta[slot]
        ev = None
        if meta.is_cuda:
            hm.copy_(torch.stack(mparts), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(meta.device))
        else:
            hm.copy_(torch.stack(mparts))
        return slot, packed, mparts, ev

    def launch_payload(self, handle):
        """deferred, second half (a step later): read the sizes the first half copied to the
        host (waiting only if that copy has not landed yet) and enqueue the payload gather on
        the current stream.  Returns a handle for finish()."""
        slot, packed, mparts, ev = handle
        if not _collectives():
            return self._handle(mparts, [packed], None, packed)
        if ev is not None:
            ev.synchronize()
        sizes = self.hmeta[slot].numpy().copy()
        pparts = self._payload(slot, packed, sizes)
        return self._handle(mparts, pparts, sizes, packed)

    def launch(self, slot, packed, total, counts, n):
        """Enqueue slot `slot`'s gathers on the current stream ("sized": after reading the
        all-gathered sizes on the host); returns a handle for finish()."""
        if self.mode == "deferred":
            return self.launch_payload(self.launch_meta(slot, packed, total, counts, n))
        if packed.shape[0] != self.rows:
            raise ValueError(f"packed has {packed.shape[0]} rows, the gather was sized for {self.rows}")
        meta = self._stage_meta(slot, total, counts, n)
        coll = _collectives()
        sizes = None
        if not coll:
            mparts, pparts = [meta], [packed]
        elif self.mode == "sized":
            mparts = self._all_gather_meta(slot, meta)
            sizes = torch.stack(mparts).cpu().numpy()  # host read: this step, every rank
            pparts = self._payload(slot, packed, sizes)
        else:
            mparts, pparts = self.mparts[slot], self.pparts[slot]
            root = self.rank == self.dst
            _gather(meta, mparts if root else None, self.dst)
            _gather(packed, pparts if root else None, self.dst)
        return self._handle(mparts, pparts, sizes, packed)

    @staticmethod
    def finish(handle):
        """On `dst`: wait for the slot's gather, then (dets_u8 [P, 40] numpy, counts numpy
        int32) in global (rank, image) order; None on other ranks (no wait).  The copies out
        run on the stream the gather was enqueued on, never behind later forwards."""
        parts, done, stream = handle
        if parts is None:
            return None
        if done is not None:
            done.synchronize()
        mparts, pparts, meta = parts
        with torch.cuda.stream(stream) if stream is not None else _nullcontext():
            if meta is None:
                meta = torch.stack(mparts).cpu().numpy()  # [world, 2 + cap]
            dets = [pparts[r][:int(meta[r, 0])] for r in range(len(mparts))]
            d = torch.cat(dets, 0).cpu().numpy()
        cnt = np.concatenate([meta[r, 2:2 + int(meta[r, 1])] for r in range(len(mparts))]).astype(np.int32)
        return d, cnt


def gather_detections(packed, total, counts, n, dst=0, mode="sized"):
    """Synchronous one-step form of DetectionGather: this rank's packed detections (packed
    [rows, 40] uint8 image-major from dnn_yolo_pack_detections, total [1] int32 valid rows,
    counts [>= n] int32 per image, n valid images) gathered to `dst`.  Returns (dets_u8
    [P, 40] numpy, counts numpy int32) in global (rank, image) order on `dst`, None
    elsewhere."""
    g = DetectionGather(counts.shape[0], packed.shape[0], packed.device, slots=1, dst=dst, mode=mode)
    return g.finish(g.launch(0, packed, total, counts, n))


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


class _HostStream(object):
    """Stand-in for a HIP stream when the runner's buffers live on the host (the CPU gloo tests
    drive the pipelined path with host tensors): work is synchronous, waits are no-ops."""
    cuda_stream = 0

    def wait_event(self, ev):
        pass


class _HostEvent(object):
    """Stand-in for a HIP event on the host path: always complete, no timing."""

    def record(self, stream=None):
        pass

    def query(self):
        return True

    def synchronize(self):
        pass

    def elapsed_time(self, other):
        return 0.0


class ShardedRunner(object):
    """Runs `compute(inp, out, n)` on this rank's shard of a global batch and gathers.

    compute   callable writing outputs for the first n frames of `inp` into `out`
    in_shape  per-frame input shape, out_shape per-frame output shape

    Pipelined form (launch_detections / finish_detections): with the default gather_mode
    "deferred", finish_detections(handle of step k) returns step k - 1's detections (None for
    the first step) — the size exchange of a step is read on the host one finish later — and
    flush_detections() returns the last step's; "sized" and "fixed" return step k's own.  A
    caller collecting results in order therefore appends every non-None finish and then the
    flush (tests/test_dist_cpu.py::test_pipelined_runner_deferred_order_gloo).
    """

    def __init__(self, compute, global_batch, in_shape, out_shape, device, dtype=torch.float32, timing=True,
                 slots=None, gather_mode="deferred", post_after=None):
        self.timing = bool(timing)  # per-step HIP timing events for stats()
        # post_after(stream_ptr) (pipelined path, optional): a step's postprocess is enqueued right
        # after the NEXT step's forward, on the post stream made to wait by post_after -- e.g. for a
        # mark inside that forward (Plan.wait_mark) -- so it runs beside the next forward's late
        # layers instead of its first ones.  The last step's is enqueued at its finish.
        self.post_after = post_after
        if gather_mode not in DetectionGather.MODES:
            raise ValueError(f"gather_mode {gather_mode!r}")
        self.gather_mode = gather_mode  # DetectionGather mode of the pipelined path
        # output / detection buffer slots of the pipelined path (launch_detections /
        # finish_detections), and steps in flight: the caller finishes step k once step
        # k + inflight - 1 has been launched.  "deferred" completes a step's gather one finish
        # later, so it holds one slot more than it keeps steps in flight
        deferred = gather_mode == "deferred"
        self.slots = int(slots) if slots is not None else (4 if deferred else 3)
        self.inflight = self.slots - 1 if deferred else self.slots
        if self.inflight < 1:
            raise ValueError(f"slots={self.slots} leaves no step in flight")
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
        """Pipelined form of step_detections, first half — nothing here waits on the host:
        the forward for this rank's shard into output slot `slot` (< slots) on the current
        stream (after the slot's previous gather has drained, device-side), then
        `post(out, n, slot, stream_ptr)` (postprocess + pack) on a post stream that waits
        only for that forward, so step k's postprocessing runs beside step k+1's first
        layers.  Returns a handle for finish_detections."""
        dev = self.out.device
        host = dev.type != "cuda"
        if not hasattr(self, "_outs"):
            self._outs = [self.out] + [torch.zeros_like(self.out) for _ in range(self.slots - 1)]
            # high-priority streams: HIP gives each its own hardware queue (GPU_MAX_HW_QUEUES
            # = 4 normal queues are shared round-robin by torch's stream pool, RCCL's internal
            # streams and the null stream; tools/stream_queue_probe.py), so neither the
            # postprocess nor the gather can end up serialised behind later forwards
            self._side = _HostStream() if host else torch.cuda.Stream(dev, priority=-1)
            self._post = _HostStream() if host else torch.cuda.Stream(dev, priority=-1)
            self._freed = [None] * self.slots
            self._gather = None
            self._deferred = None
            self._post_wait = None  # post_after: the step whose postprocess awaits the next forward
            self.reset_stats()
        cur = _HostStream() if host else torch.cuda.current_stream(dev)
        if self._freed[slot] is not None:
            cur.wait_event(self._freed[slot])
        # ev: 0/1 forward, 2 pack done, 3 gather enqueued (deferred: the size exchange), 4 gather
        # done, 5 payload gather start (deferred mode; the same point as 3 otherwise), 6 post start
        ev = [_HostEvent() if host else torch.cuda.Event(enable_timing=self.timing) for _ in range(7)]
        out = self._outs[slot]
        ev[0].record(cur)
        self.compute(local_in, out, self.count)
        ev[1].record(cur)
        h = [slot, None, None, None, ev, (out, post)]  # packed / total / counts once its post is enqueued
        if self.post_after is None:
            self._enqueue_post(h, None)
        else:
            if self._post_wait is not None:  # the previous step's, beside this forward's late layers
                self._enqueue_post(self._post_wait, None if host else self.post_after)
            self._post_wait = h
        return h

    def _enqueue_post(self, h, after):
        slot, ev = h[0], h[4]
        out, post = h[5]
        self._post.wait_event(ev[1])
        with self._on(self._post):
            if after is not None:
                after(self._post.cuda_stream)
            ev[6].record(self._post)
            h[1], h[2], h[3] = post(out, self.count, slot, self._post.cuda_stream)
            ev[2].record(self._post)
        h[5] = None

    @staticmethod
    def _on(stream):
        return _nullcontext() if isinstance(stream, _HostStream) else torch.cuda.stream(stream)

    def finish_detections(self, handle):
        """Second half, called once the next inflight - 1 steps have been launched (three by
        default, so rank 0 waits for a gather that finished a forward ago and the host never
        starves the queue while an RCCL gather waits for CUs): enqueue the detection gather
        (DetectionGather) on a side stream that waits only for this step's pack — enqueued
        this late so that no stream whose hardware queue may be shared with the run stream
        holds a wait ahead of the next forward — then on rank 0 wait for it and return
        (dets_u8 [P, 40], counts [global_batch]) numpy, None on other ranks.
        Host synchronisation by mode: "fixed" — none on non-root ranks; "sized" — every
        rank reads this step's all-gathered sizes (a wait for this step's pack on ALL ranks);
        "deferred" — this call enqueues this step's size exchange and completes the PREVIOUS
        step's gather (sizes read a step after their exchange), returning the previous
        step's detections; flush_detections() completes the last one."""
        if handle[5] is not None:  # post_after: the last step's postprocess, after its own forward
            if self._post_wait is handle:
                self._post_wait = None
            self._enqueue_post(handle, None)
        slot, packed, total, counts, ev = handle[:5]
        if self._gather is None:
            self._gather = DetectionGather(self.shard_cap, packed.shape[0], self.out.device,
                                           slots=self.slots, mode=self.gather_mode)
        t0 = time.perf_counter()
        if self.gather_mode == "deferred":
            # the previous step's payload gather first (its sizes were exchanged a step ago), so
            # it does not queue on the side stream behind this step's size exchange, which
            # waits for this step's pack; then this step's size exchange
            prev, self._deferred = self._deferred, None
            r = self._complete(prev) if prev is not None else None
            with self._on(self._side):
                self._side.wait_event(ev[2])
                ev[3].record(self._side)
                ha = self._gather.launch_meta(slot, packed, total, counts, self.count)
            self._deferred = (ha, ev, slot)
            self._host_blocked += time.perf_counter() - t0
            return r
        with self._on(self._side):
            self._side.wait_event(ev[2])
            ev[3].record(self._side)
            ev[5].record(self._side)
            gh = self._gather.launch(slot, packed, total, counts, self.count)
            ev[4].record(self._side)
        self._freed[slot] = ev[4]
        r = DetectionGather.finish(gh)
        self._host_blocked += time.perf_counter() - t0
        self._note(ev)
        return r

    def _complete(self, deferred):
        """deferred mode: the payload gather of a step whose size exchange was enqueued one
        finish earlier, then (rank 0) its detections."""
        ha, ev, slot = deferred
        with self._on(self._side):
            ev[5].record(self._side)
            gh = self._gather.launch_payload(ha)
            ev[4].record(self._side)
        self._freed[slot] = ev[4]
        r = DetectionGather.finish(gh)
        self._note(ev)
        return r

    def flush_detections(self):
        """deferred mode: complete the last step's gather (rank 0: its detections); None when
        nothing is pending or in the other modes."""
        if self.gather_mode != "deferred" or getattr(self, "_deferred", None) is None:
            return None
        t0 = time.perf_counter()
        prev, self._deferred = self._deferred, None
        r = self._complete(prev)
        self._host_blocked += time.perf_counter() - t0
        return r

    def _note(self, ev):
        """Account a finished step's events: running sums, not a growing list (a serving loop
        runs unbounded steps); events are read once complete."""
        self._evq.append(ev)
        self._account(force=False)

    def _account(self, force):
        while self._evq and (force or self._evq[0][4].query()):
            e = self._evq.pop(0)
            self._nsteps += 1
            if self.timing:
                if force:
                    e[4].synchronize()
                self._sums[0] += e[0].elapsed_time(e[1])
                self._sums[1] += e[6].elapsed_time(e[2])
                self._sums[2] += e[5].elapsed_time(e[4])
                self._sums[3] += e[3].elapsed_time(e[4])

    def reset_stats(self):
        self._evq, self._nsteps, self._sums, self._host_blocked = [], 0, [0.0, 0.0, 0.0, 0.0], 0.0
        self._deferred = getattr(self, "_deferred", None)

    def stats(self):
        """Per-step means (ms) over the steps finished since reset_stats(): forward (run
        stream), post (postprocess + pack), gather (side stream: the gather of the detections
        themselves -- in "deferred" mode the payload gather alone), gather_span (side stream,
        from the step's first gather operation to its last: in "deferred" mode from the size
        exchange to the payload gather a step later, so it spans the next step's forward),
        host_blocked (host time inside finish_detections / flush_detections).  Call after
        synchronising."""
        self._account(force=True)
        n = self._nsteps
        if n == 0 or not self.timing:
            return {"host_blocked_ms": round(self._host_blocked * 1e3 / max(n, 1), 4), "steps": n}
        f, p, g, gs = (v / n for v in self._sums)
        return {"forward_ms": round(f, 4), "post_ms": round(p, 4), "gather_ms": round(g, 4),
                "gather_span_ms": round(gs, 4), "host_blocked_ms": round(self._host_blocked * 1e3 / n, 4),
                "steps": n}

    def step_detections(self, local_in, post, mode="sized"):
        """One batch ending in detections: local compute, then `post(out, n)` -> (packed
        [rows, 40] uint8, total [1] int32, counts [cap] int32) on this rank's device (the
        on-GPU postprocessing + pack), then the packed detection gather.  Returns (dets_u8
        [P, 40], counts [global_batch]) on rank 0 (unpack_detections turns them into rows),
        None elsewhere."""
        self.compute(local_in, self.out, self.count)
        packed, total, counts = post(self.out, self.count)
        return gather_detections(packed, total, counts, self.count, mode=mode)
