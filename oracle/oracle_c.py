"""TEST INFRASTRUCTURE ONLY — ctypes binding of oracle/liboracle_dnn.so (dnn_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle_dnn.so")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    if not os.path.exists(_LIB):
        build()
    lib = ctypes.CDLL(_LIB)
    P = ctypes.c_void_p
    i, f = ctypes.c_int, ctypes.c_float
    lib.oracle_im2col.argtypes = [P, P] + [i] * 9
    lib.oracle_conv2d_mul.argtypes = [P, P, P] + [i] * 11
    lib.oracle_conv2d_direct.argtypes = [P, P, P, i, P, i]
    lib.oracle_bias_add.argtypes = [P, P, P, i, i, i, i]
    lib.oracle_batch_norm.argtypes = [P, P, P, P, f, P, i, i, i, i]
    lib.oracle_batch_norm_ab.argtypes = [P, P, P, P, i, i, i, i]
    lib.oracle_leaky_relu.argtypes = [P, P, i, i, i, i, i]
    lib.oracle_max_pool2d.argtypes = [P, P] + [i] * 13
    lib.oracle_conv2d_sgemm.argtypes = [P, P, P] + [i] * 11 + [P]
    for fn in ("oracle_im2col", "oracle_conv2d_mul", "oracle_conv2d_sgemm", "oracle_conv2d_direct", "oracle_bias_add",
               "oracle_batch_norm", "oracle_batch_norm_ab", "oracle_leaky_relu", "oracle_max_pool2d"):
        getattr(lib, fn).restype = None
    return lib


def openblas_sgemm():
    """(address of cblas_sgemm, OpenBLAS thread count) from the OpenBLAS build scipy ships
    (symbol scipy_cblas_sgemm, 32-bit ints) — the library proj3's OpenBLAS engine links
    (dnn_openblas.c:1,184-192).  None when no such build is importable."""
    import glob
    import scipy
    d = os.path.join(os.path.dirname(os.path.dirname(scipy.__file__)), "scipy.libs")
    for path in sorted(glob.glob(os.path.join(d, "libscipy_openblas-*.so"))):
        try:
            lib = ctypes.CDLL(path)
            fn = lib.scipy_cblas_sgemm
        except (OSError, AttributeError):
            continue
        nthreads = 1
        try:
            lib.scipy_openblas_get_num_threads.restype = ctypes.c_int
            nthreads = int(lib.scipy_openblas_get_num_threads())
        except AttributeError:
            pass
        _KEEP.append(lib)
        return ctypes.cast(fn, ctypes.c_void_p).value, nthreads
    return None


_KEEP = []


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleC(object):
    """numpy-friendly wrappers around the C restatement."""

    def __init__(self):
        self.lib = load()

    def conv2d_mul(self, xp, kernel_r, oh, ow, kh, kw, sh, sw):
        xp, kernel_r = _f32(xp), _f32(kernel_r)
        B, ih, iw, ic = xp.shape
        od = kernel_r.shape[1]
        out = np.empty((B, oh, ow, od), np.float32)
        self.lib.oracle_conv2d_mul(_p(xp), _p(kernel_r), _p(out), B, oh, ow, od, ih, iw, ic, kh, kw, sh, sw)
        return out

    def conv2d_sgemm(self, xp, kernel_r, oh, ow, kh, kw, sh, sw, sgemm):
        xp, kernel_r = _f32(xp), _f32(kernel_r)
        B, ih, iw, ic = xp.shape
        od = kernel_r.shape[1]
        out = np.empty((B, oh, ow, od), np.float32)
        self.lib.oracle_conv2d_sgemm(_p(xp), _p(kernel_r), _p(out), B, oh, ow, od, ih, iw, ic, kh, kw, sh, sw,
                                     ctypes.c_void_p(sgemm))
        return out

    def conv2d_direct(self, xp, kernel_hwio, oh, ow, sh, sw, nthreads=4):
        xp, k = _f32(xp), _f32(kernel_hwio)
        B, ih, iw, ic = xp.shape
        kh, kw, _, od = k.shape
        args = np.array([oh, ow, od, ih, iw, ic, kh, kw, sh, sw], np.int32)
        out = np.empty((B, oh, ow, od), np.float32)
        self.lib.oracle_conv2d_direct(_p(xp), _p(k), _p(out), B, _p(args), nthreads)
        return out

    def bias_add(self, x, b):
        x, b = _f32(x), _f32(b)
        out = np.empty_like(x)
        self.lib.oracle_bias_add(_p(x), _p(b), _p(out), *x.shape)
        return out

    def batch_norm(self, x, mean, var, gamma, eps):
        x, mean, var, gamma = _f32(x), _f32(mean), _f32(var), _f32(gamma)
        out = np.empty_like(x)
        self.lib.oracle_batch_norm(_p(x), _p(mean), _p(var), _p(gamma), float(eps), _p(out), *x.shape)
        return out

    def batch_norm_ab(self, x, alpha, beta):
        x, alpha, beta = _f32(x), _f32(alpha), _f32(beta)
        out = np.empty_like(x)
        self.lib.oracle_batch_norm_ab(_p(x), _p(alpha), _p(beta), _p(out), *x.shape)
        return out

    def leaky_relu(self, x, f32_variant=0):
        x = _f32(x)
        out = np.empty_like(x)
        self.lib.oracle_leaky_relu(_p(x), _p(out), *x.shape, int(f32_variant))
        return out

    def max_pool2d(self, x, ksize, strides, padding, gt_below=0):
        from ref_numpy import get_out_pads  # noqa: E402  (same directory)
        x = _f32(x)
        B, h, w, c = x.shape
        kh, kw, sh, sw = ksize[1], ksize[2], strides[1], strides[2]
        oh, pt, _ = get_out_pads(h, kh, sh, padding)
        ow, pl, _ = get_out_pads(w, kw, sw, padding)
        out = np.empty((B, oh, ow, c), np.float32)
        self.lib.oracle_max_pool2d(_p(x), _p(out), B, h, w, c, oh, ow, kh, kw, sh, sw, pt, pl, int(gt_below))
        return out


def openblas_kernels(weights):
    """Per conv the kernel_r the OpenBLAS engine hands conv2d_mul: HWIO transposed to
    (ic, kh, kw) rows x od columns (dnn_openblas.py:167)."""
    return [np.ascontiguousarray(w["kernel"].transpose(2, 0, 1, 3).reshape(-1, w["kernel"].shape[3]),
                                 dtype=np.float32) for w in weights]


def yolo_forward_openblas(oc, weights, x, sgemm, kernels_r=None):
    """BASELINE config 1: one YOLOv2-tiny forward through the OpenBLAS engine's per-node C
    calls (proj3/dnn_openblas.py node order): host np.pad, conv2d_mul = im2col + OpenBLAS
    cblas_sgemm (dnn_openblas.c:160-194, oracle_conv2d_sgemm), bias_add, batch_norm(mean,
    var, gamma, eps) (:40-65), leaky (:236-254) and max_pool2d over the -FLT_MAX padded input
    (:196-234, dnn_openblas.py:232-235).  CPU-baseline timing only (bench.py)."""
    from ref_numpy import pad_nhwc  # noqa: E402  (same directory)
    kr = kernels_r if kernels_r is not None else openblas_kernels(weights)
    y = _f32(x)
    last = len(weights) - 1
    for i, w in enumerate(weights):
        kh, kw = w["kernel"].shape[0], w["kernel"].shape[1]
        xp, oh, ow = pad_nhwc(y, kh, kw, 1, 1, "SAME")
        y = oc.conv2d_sgemm(xp, kr[i], oh, ow, kh, kw, 1, 1, sgemm)
        y = oc.bias_add(y, w["biases"])
        if i == last:
            break
        y = oc.batch_norm(y, w["moving_mean"], w["moving_variance"], w["gamma"], 1e-5)
        y = oc.leaky_relu(y)
        if i < 5:
            y = oc.max_pool2d(y, [1, 2, 2, 1], [1, 2, 2, 1], "SAME")
        elif i == 5:
            y = oc.max_pool2d(y, [1, 2, 2, 1], [1, 1, 1, 1], "SAME")
    return y


def yolo_forward_avx(oc, weights, x, nthreads=4):
    """The AVX engine's per-node work for one YOLOv2-tiny forward (proj3/dnn_avx.py node
    order): host pad, direct conv over `nthreads` pthreads (P_THREADS = 4, dnn_avx.c:13),
    bias_add, batch_norm in the folded alpha/beta form (dnn_avx.py:301-303), leaky max(x, 0.1x)
    and max pool.  CPU-baseline timing only (bench.py); the numerics oracle is ref_numpy."""
    from ref_numpy import pad_nhwc  # noqa: E402  (same directory)
    y = _f32(x)
    last = len(weights) - 1
    for i, w in enumerate(weights):
        k = w["kernel"]
        kh, kw = k.shape[0], k.shape[1]
        xp, oh, ow = pad_nhwc(y, kh, kw, 1, 1, "SAME")
        y = oc.conv2d_direct(xp, k, oh, ow, 1, 1, nthreads=nthreads)
        y = oc.bias_add(y, w["biases"])
        if i == last:
            break
        alpha = (w["gamma"] / np.sqrt(w["moving_variance"] + np.float32(1e-5))).astype(np.float32)
        y = oc.batch_norm_ab(y, alpha, (alpha * w["moving_mean"]).astype(np.float32))
        y = oc.leaky_relu(y, f32_variant=1)
        if i < 5:
            y = oc.max_pool2d(y, [1, 2, 2, 1], [1, 2, 2, 1], "SAME")
        elif i == 5:
            y = oc.max_pool2d(y, [1, 2, 2, 1], [1, 1, 1, 1], "SAME")
    return y
