"""Pin the oracle: the numpy and C restatements against the golden vectors produced by the
reference's own engine (cs492-projects/proj3/dnn.py, tests/golden/make_golden.py).  CPU only."""
import hashlib

import numpy as np
import pytest

import ref_numpy as R
import synth
from oracle_c import OracleC

TOL = 1e-4  # normwise parity bar of the north star

CONV_CASES = ["c3_same", "c3_same_c3", "c3_valid", "c1_same", "c2_same", "c3_wide"]
EW_CASES = ["a", "b", "c"]
POOL_CASES = ["k2s2_even", "k2s2_odd", "k2s1_same", "k3s2_valid", "k3s2_same"]


@pytest.fixture(scope="module")
def oc():
    return OracleC()


def test_generator_reproduces_spec(golden_spec):
    ws = synth.yolo_weights()
    assert synth.weights_digest(ws) == golden_spec["weights_sha256"]
    for i, h in golden_spec["frames"].items():
        assert hashlib.sha256(synth.frame(int(i)).tobytes()).hexdigest() == h


@pytest.mark.parametrize("name", CONV_CASES)
def test_conv_numpy_and_c_vs_golden(golden_ops, oc, name):
    x, k = golden_ops[f"conv_{name}_x"], golden_ops[f"conv_{name}_k"]
    pad = str(golden_ops[f"conv_{name}_pad"])
    ref = golden_ops[f"conv_{name}_y"]
    y = R.conv2d(x, k, padding=pad)
    assert y.shape == ref.shape
    assert R.normwise_err(y, ref) < 1e-6
    # C restatement of conv2d_mul: host pad + kernel_r in (ic, kh, kw) order
    kh, kw, ic, od = k.shape
    xp, oh, ow = R.pad_nhwc(x, kh, kw, 1, 1, pad)
    kr = np.ascontiguousarray(k.transpose(2, 0, 1, 3).reshape(-1, od))
    yc = oc.conv2d_mul(xp, kr, oh, ow, kh, kw, 1, 1)
    assert R.normwise_err(yc, ref) < 1e-6
    yd = oc.conv2d_direct(xp, k, oh, ow, 1, 1, nthreads=3)
    assert R.normwise_err(yd, ref) < 1e-6


@pytest.mark.parametrize("name", EW_CASES)
def test_elementwise_vs_golden(golden_ops, oc, name):
    g = golden_ops
    x = g[f"bias_{name}_x"]
    assert np.array_equal(R.bias_add(x, g[f"bias_{name}_b"]), g[f"bias_{name}_y"])
    assert np.array_equal(oc.bias_add(x, g[f"bias_{name}_b"]), g[f"bias_{name}_y"])
    bn = R.batch_norm(g[f"bn_{name}_x"], g[f"bn_{name}_mean"], g[f"bn_{name}_var"], g[f"bn_{name}_gamma"], 1e-5)
    assert np.array_equal(bn, g[f"bn_{name}_y"])
    bnc = oc.batch_norm(g[f"bn_{name}_x"], g[f"bn_{name}_mean"], g[f"bn_{name}_var"], g[f"bn_{name}_gamma"], 1e-5)
    assert np.array_equal(bnc, g[f"bn_{name}_y"])
    # dnn.py's np.vectorize leaky hands each element to the lambda as a Python float, so
    # 0.1*t is rounded in double then stored as fp32: the OpenBLAS C form bit for bit.  The
    # AVX form (0.1f*t in fp32) is at most 1 ulp away.
    xl = g[f"leaky_{name}_x"]
    assert np.array_equal(R.leaky_relu(xl), g[f"leaky_{name}_y"])
    assert np.array_equal(oc.leaky_relu(xl, 0), g[f"leaky_{name}_y"])
    d = np.abs(R.leaky_relu_avx(xl).view(np.int32).astype(np.int64) - g[f"leaky_{name}_y"].view(np.int32))
    assert d.max() <= 1
    assert np.array_equal(oc.leaky_relu(xl, 1), R.leaky_relu_avx(xl))


@pytest.mark.parametrize("name", POOL_CASES)
def test_pool_vs_golden(golden_ops, oc, name):
    g = golden_ops
    x = g[f"pool_{name}_x"]
    k, s = g[f"pool_{name}_k"], g[f"pool_{name}_s"]
    pad = str(g[f"pool_{name}_pad"])
    ks, ss = [1, int(k[0]), int(k[1]), 1], [1, int(s[0]), int(s[1]), 1]
    ref = g[f"pool_{name}_y"]
    assert np.array_equal(R.max_pool2d(x, ks, ss, pad), ref)
    assert np.array_equal(oc.max_pool2d(x, ks, ss, pad), ref)
    assert np.array_equal(oc.max_pool2d(x, ks, ss, pad, gt_below=x.shape[3]), ref)


def test_batch_norm_ab_fold_matches_mvg_within_ulps(oc):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 3, 4, 24)).astype(np.float32)
    mean = rng.uniform(-0.2, 0.2, 24).astype(np.float32)
    var = rng.uniform(0.5, 1.5, 24).astype(np.float32)
    gamma = rng.uniform(0.5, 1.5, 24).astype(np.float32)
    alpha = (gamma / np.sqrt(var + np.float32(1e-5))).astype(np.float32)  # dnn_avx.py:301-303
    beta = (alpha * mean).astype(np.float32)
    a = oc.batch_norm_ab(x, alpha, beta)
    assert np.array_equal(a, R.batch_norm_ab(x, alpha, beta))
    assert R.normwise_err(a, R.batch_norm(x, mean, var, gamma, 1e-5)) < 1e-6


def test_im2col_orders(oc):
    rng = np.random.default_rng(3)
    xp = rng.standard_normal((1, 6, 7, 5)).astype(np.float32)
    col = R.im2col(xp, 3, 3, 1, 2, 4, 3, order="ckk")[0]
    colc = np.empty_like(col)
    oc.lib.oracle_im2col(xp.ctypes.data, colc.ctypes.data, 4, 3, 6, 7, 5, 3, 3, 1, 2)
    assert np.array_equal(col, colc)


@pytest.mark.parametrize("frame", [0, 1, 2, 3])
def test_whole_net_numpy_vs_golden(golden_frames, yolo_weights, frame):
    if frame not in golden_frames:
        pytest.skip("golden frame missing")
    y = R.yolo_forward(yolo_weights, synth.frame(frame))
    err = R.normwise_err(y, golden_frames[frame])
    assert y.shape == (1, 13, 13, 125)
    assert err < 1e-5, err


def test_openblas_engine_ctypes_vs_golden(golden_frames, yolo_weights, oc):
    """BASELINE config 1 (the bench's cpu_baseline value): the OpenBLAS engine's per-node C
    calls with conv2d_mul = im2col + OpenBLAS cblas_sgemm, one frame, vs the reference golden."""
    import oracle_c
    sg = oracle_c.openblas_sgemm()
    if sg is None:
        pytest.skip("no OpenBLAS build to bind")
    y = oracle_c.yolo_forward_openblas(oc, yolo_weights, synth.frame(0), sg[0])
    assert y.shape == (1, 13, 13, 125)
    assert R.normwise_err(y, golden_frames[0]) < 1e-5


def test_node_stats_vs_golden(yolo_weights):
    import os
    from conftest import GOLDEN
    st = np.load(os.path.join(GOLDEN, "nodes_frame0.npz"))
    _, nodes = R.yolo_forward(yolo_weights, synth.frame(0), keep=True)
    assert len(nodes) == 40
    for k, r in enumerate(nodes):
        assert tuple(st[f"shape_{k}"]) == r.shape
        idx = np.linspace(0, r.size - 1, 64).astype(np.int64)
        samp = r.reshape(-1)[idx]
        assert R.normwise_err(samp, st[f"sample_{k}"]) < TOL
        assert abs(float(np.abs(r).max()) - float(st[f"maxabs_{k}"])) <= TOL * float(st[f"maxabs_{k}"])


def test_postprocessing_restatement_vs_reference_golden(post_golden):
    """oracle/post_numpy.py == the reference's own postprocessing() on every fixture case
    (dense, empty, single, ties, >64-bit IoU products, and the 4 whole-net outputs)."""
    import post_numpy as PN
    total = 0
    for name, (pred, gold) in post_golden.items():
        if isinstance(gold, dict):  # the reference raises on this input
            with pytest.raises(ZeroDivisionError):
                PN.postprocessing(pred)
            continue
        got = [[b[0], list(b[1]), list(b[2])] for b in PN.postprocessing(pred)]
        assert got == gold, name
        total += len(gold)
    assert total > 400


def test_postprocessing_restatement_edge_semantics():
    import post_numpy as PN
    # IoU has no clamp: two far-apart boxes with negative overlaps in x AND y get a positive
    # "intersection" (yolov2tiny.py:186-190)
    a, b = [0, 0, 10, 10], [100, 100, 110, 110]
    assert PN.iou(a, b) == 7921 / float(121 + 121 - 7921)
    # float32 threshold: a score equal to float32(0.3) is not kept (numpy compares in fp32)
    assert not (np.float32(0.3) > np.float32(0.3)) and (float(np.float32(0.3)) > 0.3)
