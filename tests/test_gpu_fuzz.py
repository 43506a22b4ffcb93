"""Seeded shape fuzz over the fused conv paths (implicit GEMM, fused pool, patch, direct conv0,
split-K, every tile config the chooser can reach): for random batch sizes, odd and even
spatial sizes, channel counts and epilogue variants, the fused plan must equal the explicit
im2col + GEMM + pool plan (DNN_HIP_FUSE=0) bit for bit where they share the MFMA family and
K order, and both must be within the per-layer normwise tolerance of the float64 oracle.
Shapes are kept small enough for the numpy oracle to finish in well under a second each."""
import numpy as np
import pytest

import dnn_hip
import ref_numpy as R

pytestmark = pytest.mark.gpu

LAYER_TOL = 2e-6


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    C = int(rng.choice([1, 2, 3, 16, 32, 64, 96, 128]))
    OC = int(rng.choice([16, 32, 64, 125, 128, 256]))
    if C <= 3:
        OC = 16  # conv0-like layers (direct MFMA conv0 when pooled)
    H = int(rng.integers(5, 40))
    W = int(rng.integers(5, 40))
    B = int(rng.choice([1, 2, 3, 7]))
    kh = int(rng.choice([3, 3, 3, 1]))
    pool = rng.choice(["s2", "s1", "none"], p=[0.5, 0.2, 0.3])
    epi = rng.choice(["bn", "bn_neg", "bias", "none"], p=[0.5, 0.2, 0.2, 0.1])
    return B, H, W, C, kh, OC, str(pool), str(epi), rng


def _graph(shape, k, bias, bn, leaky, pool):
    g = dnn_hip.DnnGraphBuilder()
    y = g.create_input(list(shape))
    y = g.create_conv2d(y, k, [1, 1, 1, 1], "SAME")
    if bias is not None:
        y = g.create_bias_add(y, bias)
    if bn is not None:
        y = g.create_batch_norm(y, *bn, 1e-5)
    if leaky:
        y = g.create_leaky_relu(y)
    if pool == "s2":
        y = g.create_max_pool2d(y, [1, 2, 2, 1], [1, 2, 2, 1], "SAME")
    elif pool == "s1":
        y = g.create_max_pool2d(y, [1, 2, 2, 1], [1, 1, 1, 1], "SAME")
    g.set_out_node(y)
    return g


@pytest.mark.parametrize("seed", range(48))
def test_fused_plan_shape_fuzz(monkeypatch, seed):
    B, H, W, C, kh, OC, pool, epi, rng = _case(seed)
    x = rng.standard_normal((B, H, W, C)).astype(np.float32)
    k = (rng.standard_normal((kh, kh, C, OC)) * np.sqrt(2.0 / (kh * kh * C))).astype(np.float32)
    bias = (rng.standard_normal(OC) * 0.1).astype(np.float32) if epi != "none" else None
    bn = None
    if epi.startswith("bn"):
        gamma = rng.uniform(0.5, 1.5, OC).astype(np.float32)
        if epi == "bn_neg":
            gamma[::2] *= -1.0  # non-increasing epilogue channels: min-pool before the epilogue
        bn = ((rng.standard_normal(OC) * 0.1).astype(np.float32), rng.uniform(0.5, 1.5, OC).astype(np.float32), gamma)
    leaky = epi != "none"

    outs, descs = {}, {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("DNN_HIP_FUSE", fuse)
        eng = dnn_hip.DnnInferenceEngine(_graph(x.shape, k, bias, bn, leaky, pool), False)
        outs[fuse] = eng.run(x)
        descs[fuse] = eng.plan().describe()

    ref = R.conv2d(x, k, strides=(1, 1, 1, 1), padding="SAME")
    if bias is not None:
        ref = R.bias_add(ref, bias)
    if bn is not None:
        ref = R.batch_norm(ref, *bn, 1e-5)
    if leaky:
        ref = R.leaky_relu(ref)
    if pool == "s2":
        ref = R.max_pool2d(ref, [1, 2, 2, 1], [1, 2, 2, 1], "SAME")
    elif pool == "s1":
        ref = R.max_pool2d(ref, [1, 2, 2, 1], [1, 1, 1, 1], "SAME")
    info = f"case B={B} H={H} W={W} C={C} k={kh} OC={OC} pool={pool} epi={epi}\n{descs['1']}"
    assert outs["1"].shape == ref.shape, info
    for fuse in ("1", "0"):
        assert np.all(np.isfinite(outs[fuse])), info
        assert R.normwise_err(outs[fuse], ref) < LAYER_TOL, info + f"\nfuse={fuse}"
    # fused vs explicit: bit-exact when both run the same MFMA family and K order (the GEMM
    # paths); the patch / direct conv kernels use their own tap order and are held to the
    # oracle bar above
    if "mode=implicit" in descs["1"] or "mode=gemm" in descs["1"] or "mode=direct_a" in descs["1"]:
        assert np.array_equal(outs["1"], outs["0"]), info
