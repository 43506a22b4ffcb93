import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dnn-inference-engine_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _ensure_built():
    libs = [os.path.join(PKG, "libdnn_hip.so"), os.path.join(PKG, "libdnn_hip_avx.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(PKG, "csrc")], check=True)
    if not os.path.exists(os.path.join(ORACLE, "liboracle_dnn.so")):
        subprocess.run(["make", "-s", "-C", ORACLE], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_ops():
    return dict(np.load(os.path.join(GOLDEN, "ops.npz")))


@pytest.fixture(scope="session")
def golden_spec():
    with open(os.path.join(GOLDEN, "spec.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_frames():
    out = {}
    for i in range(4):
        p = os.path.join(GOLDEN, f"net_frame{i}.npy")
        if os.path.exists(p):
            out[i] = np.load(p)
    return out


@pytest.fixture(scope="session")
def yolo_weights():
    import synth
    return synth.yolo_weights()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def post_golden():
    """Postprocessing fixtures (tests/golden/make_golden_post.py): name -> (pred [13,13,125],
    reference label_boxes as [name, [l, t], [r, b]])."""
    with open(os.path.join(GOLDEN, "post_golden.json")) as f:
        gold = json.load(f)["cases"]
    d = np.load(os.path.join(GOLDEN, "post_cases.npz"))
    preds = dict(zip([str(n) for n in d["names"]], d["preds"]))
    for i in range(4):
        preds[f"net_frame{i}"] = np.load(os.path.join(GOLDEN, f"net_frame{i}.npy")).reshape(13, 13, 125)
    assert sorted(preds) == sorted(gold)
    return {k: (preds[k], gold[k]) for k in sorted(gold)}
