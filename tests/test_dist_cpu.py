"""The N>1 path on CPU: world_size-2 and world_size-8 gloo processes drive dist.py exactly as
bench.py does on RCCL — weights broadcast once from rank 0, each rank computes its contiguous
shard, outputs (or the packed detections, both DetectionGather modes) gathered to rank 0 — with the numpy
oracle standing in for the HIP plan.  Ragged global batches include ranks with no frames."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ORACLE, PKG, REPO

import dist as D


def test_shard_range_partitions():
    for total in (0, 1, 7, 64, 512, 513):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                s, c = D.shard_range(total, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))
            counts = [D.shard_range(total, world, r)[1] for r in range(world)]
            assert max(counts) - min(counts) <= 1
    with pytest.raises(ValueError):
        D.shard_range(8, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    for p in (REPO, PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import dist as Dw
    import ref_numpy as R
    Dw.init("gloo")
    try:
        rng = np.random.default_rng(5)
        k_true = rng.standard_normal((3, 3, 4, 6)).astype(np.float32)
        frames = rng.standard_normal((total, 9, 7, 4)).astype(np.float32)
        # only rank 0 holds the real weights; the others start from garbage
        w = torch.from_numpy(k_true.copy()) if rank == 0 else torch.full(k_true.shape, float(rank))
        Dw.broadcast_weights(w)
        kern = w.numpy()

        def compute(inp, out, n):
            if n:
                out[:n] = torch.from_numpy(R.conv2d(inp[:n].numpy(), kern, padding="SAME"))

        runner = Dw.ShardedRunner(compute, total, (9, 7, 4), (9, 7, 6), device="cpu")
        local = torch.from_numpy(runner.local_slice(frames))
        full = runner.step(local)
        if rank == 0:
            expect = R.conv2d(frames, k_true, padding="SAME")
            q.put(("ok", float(np.abs(full.numpy() - expect).max()), tuple(full.shape)))
        else:
            q.put(("ok", None, None))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), None))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 6), (2, 5), (8, 13), (8, 5)])
def test_sharded_broadcast_gather_gloo(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    root = [r for r in res if r[1] is not None][0]
    assert root[2] == (total, 9, 7, 6)
    assert root[1] == 0.0


def _det_worker(rank, world, port, total, q, mode):
    for p in (REPO, PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import dist as Dw
    import post_numpy as PN
    Dw.init("gloo")
    try:
        rng = np.random.default_rng(11)
        preds = np.stack([PN.synthetic_predictions(rng, n_hot=(i * 7) % 40) for i in range(total)])
        max_det = 64

        def compute(inp, out, n):  # the "network": predictions are the input frames
            out[:n] = inp[:n]

        def post(out, n):  # CPU stand-in for dnn_yolo_postprocess + pack: same packed layout
            packed = np.zeros(out.shape[0] * max_det, Dw.DETECTION_DTYPE)
            counts = np.zeros(out.shape[0], np.int32)
            p = 0
            for i in range(n):
                rows = PN.detect(out[i].numpy())
                counts[i] = len(rows)
                for (c, l, t, r, b, sc) in rows:
                    packed[p] = (c, sc, l, t, r, b)
                    p += 1
            return (torch.from_numpy(packed.view(np.uint8).reshape(-1, 40)), torch.tensor([p], dtype=torch.int32),
                    torch.from_numpy(counts))

        runner = Dw.ShardedRunner(compute, total, (13, 13, 125), (13, 13, 125), device="cpu")
        g = runner.step_detections(torch.from_numpy(runner.local_slice(preds)), post, mode=mode)
        if rank == 0:
            got = Dw.unpack_detections(*g)
            expect = [[(c, l, t, r, b, float(np.float32(sc))) for c, l, t, r, b, sc in PN.detect(p)] for p in preds]
            q.put(("ok", got == expect, sum(len(e) for e in expect)))
        else:
            q.put(("ok", None, g is None))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e), None))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,total,mode", [(2, 6, "sized"), (2, 5, "fixed"), (8, 19, "sized"), (8, 6, "sized"),
                                              (8, 13, "fixed"), (2, 7, "deferred"), (8, 19, "deferred")])
def test_sharded_detection_gather_gloo(world, total, mode):
    """Per-rank postprocessing + packed detection gather (dist.DetectionGather, all modes)
    gives rank 0 every image's detections in global order, with unequal per-rank detection
    counts, ragged shards and (8, 6) ranks that hold no image at all."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_det_worker, args=(r, world, port, total, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    root = [r for r in res if r[1] is not None][0]
    assert root[1] is True and root[2] > 10
    others = [r for r in res if r[1] is None]
    assert len(others) == world - 1 and all(r[2] is True for r in others)


def _pipe_worker(rank, world, port, total, steps, q, defer_post=False):
    for p in (REPO, PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import dist as Dw
    import post_numpy as PN
    Dw.init("gloo")
    try:
        max_det = 64
        batches = []
        for k in range(steps):
            rng = np.random.default_rng(100 + k)
            batches.append(np.stack([PN.synthetic_predictions(rng, n_hot=(i * 5 + k * 3) % 40) for i in range(total)]))

        def compute(inp, out, n):
            out[:n] = inp[:n]

        def post(out, n, slot, stream_ptr):  # the pipelined post signature (bench.py: the HIP post + pack)
            packed = np.zeros(out.shape[0] * max_det, Dw.DETECTION_DTYPE)
            counts = np.zeros(out.shape[0], np.int32)
            p = 0
            for i in range(n):
                rows = PN.detect(out[i].numpy())
                counts[i] = len(rows)
                for (c, l, t, r, b, sc) in rows:
                    packed[p] = (c, sc, l, t, r, b)
                    p += 1
            return (torch.from_numpy(packed.view(np.uint8).reshape(-1, 40)), torch.tensor([p], dtype=torch.int32),
                    torch.from_numpy(counts))

        runner = Dw.ShardedRunner(compute, total, (13, 13, 125), (13, 13, 125), device="cpu",
                                  post_after=(lambda stream: None) if defer_post else None)
        assert runner.gather_mode == "deferred" and runner.inflight == runner.slots - 1
        pending, got, firsts = [], [], []
        for k in range(steps):  # bench.py's loop: finish step k - inflight + 1 after launching step k
            pending.append(runner.launch_detections(torch.from_numpy(runner.local_slice(batches[k])), post,
                                                    k % runner.slots))
            if len(pending) == runner.inflight:
                r = runner.finish_detections(pending.pop(0))
                firsts.append(r is None)
                if r is not None:
                    got.append(r)
        while pending:
            r = runner.finish_detections(pending.pop(0))
            firsts.append(r is None)
            if r is not None:
                got.append(r)
        r = runner.flush_detections()
        if r is not None:
            got.append(r)
        if rank == 0:
            expect = [[[(c, l, t, rr, b, float(np.float32(sc))) for c, l, t, rr, b, sc in PN.detect(p)] for p in bt]
                      for bt in batches]
            q.put(("ok", [Dw.unpack_detections(*g) for g in got] == expect, (len(got), firsts[0], sum(firsts))))
        else:
            q.put(("ok", None, (len(got), sum(firsts))))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc(), None))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,total,steps,defer_post", [(2, 7, 6, False), (8, 11, 5, False), (2, 7, 6, True),
                                                         (8, 11, 5, True), (2, 5, 1, True)])
def test_pipelined_runner_deferred_order_gloo(world, total, steps, defer_post):
    """ShardedRunner's pipelined path with its default gather ("deferred"): driven as
    bench.py drives it (launch step k into slot k % slots, finish the oldest once `inflight` steps
    are pending, then drain and flush), rank 0 receives every step's detections exactly once and
    in step order: the first finish returns nothing (its sizes are read one finish later) and
    flush_detections() returns the last step; non-root ranks receive nothing.  defer_post: each
    step's postprocess enqueued after the next step's forward (post_after, bench.py's default),
    the last one at its finish -- the same detections in the same order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, total, steps, q, defer_post)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    root = [r for r in res if r[1] is not None][0]
    assert root[1] is True
    n_got, first_none, n_none = root[2]
    assert n_got == steps and first_none and n_none == 1
    others = [r for r in res if r[1] is None]
    assert len(others) == world - 1 and all(r[2] == (0, steps) for r in others)
