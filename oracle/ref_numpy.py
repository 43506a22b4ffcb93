"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's proj3 algorithms.

Used by tests/ (parity checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg;
never by the product path.  Pinned by tests/golden/* (outputs of the reference's own
cs492-projects/proj3/dnn.py, see tests/golden/make_golden.py) in
tests/test_oracle_golden.py.

Element-wise ops reproduce the reference's fp32 rounding exactly; conv accumulates in a
caller-chosen dtype (float64 gives a tighter reference than the reference itself).
"""
import math

import numpy as np

F32_MIN = np.finfo(np.float32).min


def get_out_pads(in_size, filter_size, stride_size, padding):
    """proj3/dnn_openblas.py:127-142 (TF SAME / VALID)."""
    if padding == "SAME":
        out_size = math.ceil(float(in_size) / float(stride_size))
        pad = max((out_size - 1) * stride_size + filter_size - in_size, 0)
        return out_size, pad // 2, pad - pad // 2
    out_size = math.ceil(float(in_size - filter_size + 1) / float(stride_size))
    return out_size, 0, 0


def pad_nhwc(x, kh, kw, sh, sw, padding, value=0.0):
    oh, pt, pb = get_out_pads(x.shape[1], kh, sh, padding)
    ow, pl, pr = get_out_pads(x.shape[2], kw, sw, padding)
    xp = np.pad(x, [(0, 0), (pt, pb), (pl, pr), (0, 0)], "constant", constant_values=value)
    return xp, oh, ow


def im2col(xp, kh, kw, sh, sw, oh, ow, order="ckk"):
    """proj3/dnn_openblas.c:135-158 on a padded batch: [B, oh*ow, K].
    order "ckk": K = (c, kh, kw) as the reference; "kkc": K = (kh, kw, c)."""
    B, _, _, C = xp.shape
    cols = np.empty((B, oh, ow, kh, kw, C), dtype=xp.dtype)
    for di in range(kh):
        for dj in range(kw):
            cols[:, :, :, di, dj, :] = xp[:, di:di + sh * (oh - 1) + 1:sh, dj:dj + sw * (ow - 1) + 1:sw, :]
    if order == "ckk":
        cols = cols.transpose(0, 1, 2, 5, 3, 4)
    return cols.reshape(B, oh * ow, -1)


def conv2d(x, kernel, strides=(1, 1, 1, 1), padding="SAME", acc=np.float64):
    """Conv2D node (proj3/dnn.py:168-207 semantics; im2col + GEMM as dnn_openblas.c:160-194).
    x NHWC, kernel HWIO; returns fp32 NHWC."""
    kh, kw, ic, od = kernel.shape
    sh, sw = strides[1], strides[2]
    xp, oh, ow = pad_nhwc(np.asarray(x, np.float32), kh, kw, sh, sw, padding)
    col = im2col(xp, kh, kw, sh, sw, oh, ow, order="kkc").astype(acc)
    w = np.asarray(kernel, np.float32).reshape(kh * kw * ic, od).astype(acc)
    y = col @ w
    return y.reshape(x.shape[0], oh, ow, od).astype(np.float32)


def bias_add(x, b):
    """proj3/dnn_openblas.c:9-38 / dnn.py:250."""
    return (np.asarray(x, np.float32) + np.asarray(b, np.float32)).astype(np.float32)


def batch_norm(x, mean, var, gamma, eps):
    """proj3/dnn_openblas.c:40-65 / dnn.py:324-328: ((x - mean) / sqrtf(var + eps)) * gamma, fp32."""
    sq = np.sqrt(np.asarray(var, np.float32) + np.float32(eps)).astype(np.float32)
    x = np.asarray(x, np.float32)
    return (((x - np.asarray(mean, np.float32)) / sq) * np.asarray(gamma, np.float32)).astype(np.float32)


def batch_norm_ab(x, alpha, beta):
    """proj3/dnn_avx.c:483-518: x * alpha - beta (two fp32 roundings)."""
    r = (np.asarray(x, np.float32) * np.asarray(alpha, np.float32)).astype(np.float32)
    return (r - np.asarray(beta, np.float32)).astype(np.float32)


def leaky_relu(x):
    """proj3/dnn_openblas.c:236-254: t < 0 ? (float)(0.1 * (double)t) : t."""
    x = np.asarray(x, np.float32)
    return np.where(x < 0, (0.1 * x.astype(np.float64)).astype(np.float32), x)


def leaky_relu_avx(x):
    """proj3/dnn_avx.c:525-553: _mm256_max_ps(t, 0.1f*t) = t > s ? t : s."""
    x = np.asarray(x, np.float32)
    s = (x * np.float32(0.1)).astype(np.float32)
    return np.where(x > s, x, s)


def max_pool2d(x, ksize, strides, padding, gt_below=0):
    """proj3/dnn_openblas.c:196-234 over the -FLT_MAX padded input of dnn_openblas.py:232-235:
    m = first; m = m >= v ? m : v (channels < gt_below: m > v ? m : v, _mm256_max_ps)."""
    kh, kw = ksize[1], ksize[2]
    sh, sw = strides[1], strides[2]
    xp, oh, ow = pad_nhwc(np.asarray(x, np.float32), kh, kw, sh, sw, padding, value=F32_MIN)
    win = lambda di, dj: xp[:, di:di + sh * (oh - 1) + 1:sh, dj:dj + sw * (ow - 1) + 1:sw, :]
    m = win(0, 0).copy()
    gt = np.arange(x.shape[3]) < gt_below
    for di in range(kh):
        for dj in range(kw):
            v = win(di, dj)
            m = np.where(gt, np.where(m > v, m, v), np.where(m >= v, m, v))
    return m.astype(np.float32)


def yolo_forward(weights, x, acc=np.float64, keep=False):
    """Whole YOLOv2-tiny chain (node order of proj3/yolov2tiny.py:28-79).  Returns the
    final output, or (output, [40 node results]) with keep=True."""
    nodes = []
    y = np.asarray(x, np.float32)
    last = len(weights) - 1
    for i, w in enumerate(weights):
        y = conv2d(y, w["kernel"], padding="SAME", acc=acc); nodes.append(y)
        y = bias_add(y, w["biases"]); nodes.append(y)
        if i == last:
            break
        y = batch_norm(y, w["moving_mean"], w["moving_variance"], w["gamma"], 1e-5); nodes.append(y)
        y = leaky_relu(y); nodes.append(y)
        if i < 5:
            y = max_pool2d(y, [1, 2, 2, 1], [1, 2, 2, 1], "SAME"); nodes.append(y)
        elif i == 5:
            y = max_pool2d(y, [1, 2, 2, 1], [1, 1, 1, 1], "SAME"); nodes.append(y)
    return (y, nodes) if keep else y


def normwise_err(got, ref):
    """max|got - ref| / max|ref| — the parity metric."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    denom = max(np.abs(ref).max(), 1e-30)
    return float(np.abs(got - ref).max() / denom)
