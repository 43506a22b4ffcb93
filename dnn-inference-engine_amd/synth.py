"""Portable, bit-reproducible synthetic weights and frames for YOLOv2-tiny.

The reference's weights pickle (`proj3/yolov2tiny.py:15-23`, `../y2t_weights.pickle`)
is not in the reference repo, so every test and benchmark runs on synthetic data
(SURVEY.md §8d).  The generator uses only exact integer arithmetic plus correctly
rounded IEEE operations (add, multiply, sqrt), so the same bytes come out on any
machine and any numpy version: the GPU box regenerates the 63.5 MB of weights
that the golden fixtures were computed from without shipping them.

Generator spec (also written into tests/golden/spec.json):
  * stream key   k = mix64(seed * 0x100000001B3 + stream_id)
  * raw draw  x[i] = mix64(k + (i + 1) * 0x9E3779B97F4A7C15)   (splitmix64 finaliser)
  * uniform   u[i] = (x[i] >> 40) * 2**-24                       (exact in fp32)
  * approx-normal  n[i] = (u[4i] + u[4i+1] + u[4i+2] + u[4i+3] - 2) * sqrt(3)
                                                                  (Irwin-Hall, mean 0, var 1)
Layer parameters (stream ids 10*L + j):
  kernel  HWIO  n * sqrt(2 / (kh*kw*ic))      (He-normal-like)
  biases        n * 0.1
  mean          n * 0.1
  variance      0.5 + u
  gamma         0.5 + u
Frames: uniform [0, 1) NHWC 416x416x3, seed 1 + frame index, stream 0.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

# tiny-yolo-voc channel plan; the final 125 is pinned by
# proj3/yolov2tiny.py:120 (13x13x5x25), the rest is the standard VOC plan.
CHANNELS = (16, 32, 64, 128, 256, 512, 1024, 1024, 125)
IN_SHAPE = (416, 416, 3)
WEIGHT_SEED = 0


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    return z


def _key(seed, stream):
    with np.errstate(over="ignore"):
        return _mix64(np.uint64(seed) * np.uint64(0x100000001B3) + np.uint64(stream))


def uniform(seed, stream, n, chunk=1 << 23):
    """n uniform draws in [0, 1) as float64 (each exactly representable in fp32)."""
    key = _key(seed, stream)
    out = np.empty(n, dtype=np.float64)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        idx = np.arange(s + 1, e + 1, dtype=np.uint64)
        with np.errstate(over="ignore"):
            x = _mix64(key + idx * GOLDEN)
        out[s:e] = (x >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)
    return out


def normal(seed, stream, n):
    u = uniform(seed, stream, 4 * n).reshape(n, 4)
    # left-to-right adds of 24-bit fractions are exact in float64
    s = ((u[:, 0] + u[:, 1]) + u[:, 2]) + u[:, 3]
    return (s - 2.0) * np.sqrt(3.0)


def layer_weights(layer, ic, od, k=3, seed=WEIGHT_SEED, bn=True):
    """One conv layer's parameters in the pickle's dict format
    (`proj3/yolov2tiny.py:30-77`: kernel HWIO, biases, moving_mean,
    moving_variance, gamma), fp32."""
    base = 10 * layer
    fan_in = k * k * ic
    w = {
        "kernel": (normal(seed, base + 0, k * k * ic * od) * np.sqrt(2.0 / fan_in))
        .astype(np.float32).reshape(k, k, ic, od),
        "biases": (normal(seed, base + 1, od) * 0.1).astype(np.float32),
    }
    if bn:
        w["moving_mean"] = (normal(seed, base + 2, od) * 0.1).astype(np.float32)
        w["moving_variance"] = (0.5 + uniform(seed, base + 3, od)).astype(np.float32)
        w["gamma"] = (0.5 + uniform(seed, base + 4, od)).astype(np.float32)
    return w


def yolo_weights(seed=WEIGHT_SEED, channels=CHANNELS, in_c=IN_SHAPE[2]):
    """The 9-entry weight list `build_graph` consumes (`proj3/yolov2tiny.py:26`)."""
    ws = []
    ic = in_c
    for i, od in enumerate(channels):
        last = i == len(channels) - 1
        ws.append(layer_weights(i, ic, od, k=1 if last else 3, seed=seed, bn=not last))
        ic = od
    return ws


def yolo_zero_weights(channels=CHANNELS, in_c=IN_SHAPE[2]):
    """yolo_weights' shapes with zero values, without running the generator: what a
    non-root rank lays its plan out with before the weight broadcast fills it."""
    ws, ic = [], in_c
    for i, od in enumerate(channels):
        last = i == len(channels) - 1
        k = 1 if last else 3
        w = {"kernel": np.zeros((k, k, ic, od), np.float32), "biases": np.zeros(od, np.float32)}
        if not last:
            for key in ("moving_mean", "moving_variance", "gamma"):
                w[key] = np.zeros(od, np.float32)
        ws.append(w)
        ic = od
    return ws


def frame(index, shape=IN_SHAPE):
    """Synthetic frame `index`: uniform [0,1) fp32 NHWC [1,H,W,C]
    (the range of `proj3/__init__.py:8-12` resize_input output)."""
    n = int(np.prod(shape))
    return uniform(1 + index, 0, n).astype(np.float32).reshape((1,) + tuple(shape))


def frames(indices, shape=IN_SHAPE):
    return np.concatenate([frame(i, shape) for i in indices], axis=0)


def weights_digest(ws):
    import hashlib
    h = hashlib.sha256()
    for w in ws:
        for key in ("kernel", "biases", "moving_mean", "moving_variance", "gamma"):
            if key in w:
                h.update(np.ascontiguousarray(w[key]).tobytes())
    return h.hexdigest()
