"""The N>1 bench path on a one-GPU box: `bench.py --gpus 2` relaunches itself under
torch.distributed.run, both ranks on cuda:0 with gloo (host-staged collectives) standing in
for RCCL (DNN_BENCH_SHARED_GPU / DNN_BENCH_BACKEND, rehearsal switches only): weight
broadcast, contiguous shards, on-GPU postprocessing, packed detection gather to rank 0 and
the max-over-ranks timing all run on the device path.  The 8-GPU RCCL run is the driver's."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["detections", "outputs"])
def test_bench_two_ranks_one_gpu(gather):
    env = dict(os.environ, DNN_BENCH_SHARED_GPU="1", DNN_BENCH_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--batch", "8", "--steps", "2",
           "--warmup", "1", "--no-cpu", "--no-latency", "--no-e2e", "--no-fp16", "--no-unfused", "--gather", gather]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16 and d["config"]["parallelism"] == "dp2"
    assert d["dist_backend"] == "gloo" and d["scaling"] == "weak" and d["value"] > 0
    assert d["cpu_baseline"] is None  # rank-0, N=1 only
    if gather == "detections":
        assert d["postprocess"]["detections_last_step"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["deferred", "sized"])
def test_bench_eight_ranks_one_gpu(mode):
    """BASELINE config 4's process layout rehearsed on one GPU: `bench.py --gpus 8` relaunches
    under torch.distributed.run with 8 ranks, each laying out its own device plan (batch 4:
    the shard), receiving the weight arena by broadcast, postprocessing on the device and
    gathering packed detections to rank 0 in the given gather mode; gloo host-staged
    collectives stand in for RCCL (one card).  The JSON line carries all 8 ranks."""
    env = dict(os.environ, DNN_BENCH_SHARED_GPU="1", DNN_BENCH_BACKEND="gloo", DNN_BENCH_GATHER_MODE=mode)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--batch", "4", "--steps", "4",
           "--warmup", "2", "--no-cpu", "--no-latency", "--no-e2e", "--no-fp16", "--no-unfused"]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 32 and d["config"]["parallelism"] == "dp8"
    assert len(d["per_rank"]) == 8 and [p["rank"] for p in d["per_rank"]] == list(range(8))
    assert all(p["wall_ms"] > 0 and p["forward_ms"] > 0 for p in d["per_rank"])
    assert d["postprocess"]["detections_last_step"] > 0


def _torchrun(script_args, timeout=300):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(port)] + script_args
    return subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_rccl_world1_broadcast_and_gathers():
    """A real RCCL process group (backend "nccl", world size 1, cuda:0): the weight-arena
    broadcast, gather_outputs and the pipelined detection gather (all three modes, six steps
    through every output slot; "deferred" completes each step one finish later and the last
    by flush_detections) all execute on MI355X and agree with the same work done without a
    process group."""
    r = _torchrun([os.path.join(REPO, "tests", "rccl_world1_job.py")])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["arena_ok"] and d["detections"] > 0
    assert d["outputs_shape"] == [8, 13, 13, 125]
    for mode in ("sized", "fixed", "deferred"):
        m = d["modes"][mode]
        assert m["ok"] and m["steps"] == 6, (mode, m)
        assert m["stats"]["steps"] == 6 and m["stats"]["forward_ms"] > 0


@pytest.mark.gpu
def test_bench_under_torchrun_world1_rccl():
    """bench.py as the driver launches it for N > 1 (torch.distributed.run), at one rank:
    RCCL group, broadcast, detection gathers and the per-rank breakdown in the JSON line."""
    r = _torchrun([os.path.join(REPO, "bench.py"), "--gpus", "1", "--batch", "8", "--steps", "3", "--warmup", "1",
                   "--no-cpu", "--no-latency", "--no-e2e", "--no-fp16", "--no-unfused"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["dist_backend"] == "rccl" and d["n_gpus"] == 1
    pr = d["per_rank"]
    assert len(pr) == 1 and pr[0]["forward_ms"] > 0 and pr[0]["gather_ms"] >= 0
    assert d["postprocess"]["detections_last_step"] > 0


@pytest.mark.gpu
def test_bench_eight_ranks_batch64_detections_match_single_process(tmp_path):
    """BASELINE config 4 at its real per-rank batch, rehearsed on one GPU: `bench.py --gpus 8
    --batch 64` (8 ranks x 64 frames = 512, each rank's own device plan, weight arena by
    broadcast, on-GPU postprocessing, packed detections gathered to rank 0; gloo host-staged
    collectives stand in for RCCL).  Rank 0's gathered detections of the last step equal, byte
    for byte, a single process running the same 512 frames (the ranks' seeded frames) through
    one batch-64 plan shard by shard, postprocessing and packing each shard: batch rows are
    bit-identical whatever the shard, and the gather keeps (rank, image) order."""
    import numpy as np
    import torch

    import dnn_hip
    import synth
    import yolo_graph
    import yolo_post
    dump = str(tmp_path / "dets.npz")
    env = dict(os.environ, DNN_BENCH_SHARED_GPU="1", DNN_BENCH_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--batch", "64", "--steps", "2",
           "--warmup", "1", "--preheat", "0", "--sustained", "0", "--no-cpu", "--no-latency", "--no-e2e",
           "--no-fp16", "--no-unfused", "--no-fp32-mfma", "--dump-detections", dump]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 512 and len(d["per_rank"]) == 8
    got = np.load(dump)
    assert got["counts"].shape == (512,)

    dev = torch.device("cuda", 0)
    B = 64
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(B, 416, 416, 3))
    plan = dnn_hip.Plan.from_graph(g, device=0)
    out = torch.empty((B, 13, 13, 125), device=dev)
    db = yolo_post.DetectionBuffers(B, dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    dets, counts = [], []
    for rank in range(8):
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)  # bench.py's frames of this rank
        frames = torch.rand((B, 416, 416, 3), generator=gen, device=dev, dtype=torch.float32)
        plan.run_device(B, frames.data_ptr(), out.data_ptr(), s)
        db.run(out.data_ptr(), B, s)
        packed, total, cnt = db.pack(B, s)
        torch.cuda.synchronize()
        dets.append(packed[:int(total.item())].cpu().numpy())
        counts.append(cnt[:B].cpu().numpy())
    plan.close()
    want_d, want_c = np.concatenate(dets, 0), np.concatenate(counts).astype(np.int32)
    assert np.array_equal(got["counts"], want_c)
    assert int(np.clip(want_c, 0, None).sum()) > 0 and got["dets"].shape == want_d.shape
    assert got["dets"].tobytes() == want_d.tobytes()
