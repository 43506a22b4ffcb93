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
