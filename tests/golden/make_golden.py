"""Generate the parity fixtures under tests/golden/ from the REFERENCE's own numpy engine.

Run in the build container only (it reads /root/reference, which never exists on the
GPU box):   python tests/golden/make_golden.py [--frames 4]

What it does
  * imports `cs492-projects/proj3/dnn.py` (the reference's pure numpy/scipy engine,
    SURVEY.md §2 #9, correct batched semantics) straight from /root/reference;
  * builds the YOLOv2-tiny node chain exactly as `proj3/yolov2tiny.py:28-79` lists it
    (conv, bias, bn, leaky [, pool]) with the portable synthetic weights of synth.py;
  * runs one FRESH graph per frame (dnn.py's Conv2D.run accumulates into its
    preallocated result, `proj3/dnn.py:202-207`, so a graph is single-use);
  * writes   net_frame{i}.npy      final [1,13,13,125] fp32 output per frame
             nodes_frame0.npz      per-node stats of all 40 nodes for frame 0
             ops.npz               small per-op cases through the reference node classes
             spec.json             generator spec, shapes, weight / frame SHA-256.
Only data (inputs and expected outputs) is written; no reference source is copied.
"""
import argparse
import hashlib
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "dnn-inference-engine_amd"))
import synth  # noqa: E402

REF_PROJ3 = "/root/reference/cs492-projects/proj3"


def load_reference_numpy_engine():
    spec = importlib.util.spec_from_file_location("ref_proj3_dnn", os.path.join(REF_PROJ3, "dnn.py"))
    mod = importlib.util.module_from_spec(spec)
    # dnn.py's MaxPool2D pickles its worker function into a multiprocessing.Pool
    # (proj3/dnn.py:283-301): the module must be findable by name.
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


def build_yolo(ref, weights, in_shape):
    """Node chain of proj3/yolov2tiny.py:28-79 (same order, same hyper-parameters)."""
    g = ref.DnnGraphBuilder()
    nodes = []
    x = g.create_input(in_shape)
    s1 = [1, 1, 1, 1]
    for i, w in enumerate(weights):
        x = g.create_conv2d(x, w["kernel"], strides=s1, padding="SAME"); nodes.append(x)
        x = g.create_bias_add(x, w["biases"]); nodes.append(x)
        if i == len(weights) - 1:
            break
        x = g.create_batch_norm(x, w["moving_mean"], w["moving_variance"], w["gamma"], 1e-5); nodes.append(x)
        x = g.create_leaky_relu(x); nodes.append(x)
        if i < 5:
            x = g.create_max_pool2d(x, ksize=[1, 2, 2, 1], strides=[1, 2, 2, 1], padding="SAME"); nodes.append(x)
        elif i == 5:
            x = g.create_max_pool2d(x, ksize=[1, 2, 2, 1], strides=[1, 1, 1, 1], padding="SAME"); nodes.append(x)
    g.set_out_node(x)
    return g, nodes


SAMPLE_N = 64


def sample_idx(size):
    return np.linspace(0, size - 1, SAMPLE_N).astype(np.int64)


def node_stats(nodes):
    out = {}
    for k, n in enumerate(nodes):
        r = np.asarray(n.result, dtype=np.float32)
        f = r.reshape(-1).astype(np.float64)
        out[f"shape_{k}"] = np.array(r.shape, dtype=np.int64)
        out[f"sum_{k}"] = np.array(f.sum())
        out[f"sumsq_{k}"] = np.array((f * f).sum())
        out[f"maxabs_{k}"] = np.array(np.abs(f).max())
        out[f"sample_{k}"] = r.reshape(-1)[sample_idx(r.size)]
    out["names"] = np.array([type(n).__name__ for n in nodes])
    return out


class _Fake:
    def __init__(self, arr):
        self.result = arr


def op_cases(ref):
    """Small per-op cases computed by the reference node classes (proj3/dnn.py:168-372)."""
    rng = np.random.default_rng(1234)
    cases = {}

    def f32(*shape, lo=-1.0, hi=1.0):
        return rng.uniform(lo, hi, size=shape).astype(np.float32)

    conv_cases = [
        # name, B, H, W, C, kh, kw, od, padding
        ("c3_same", 2, 7, 9, 5, 3, 3, 6, "SAME"),
        ("c3_same_c3", 1, 12, 10, 3, 3, 3, 16, "SAME"),
        ("c3_valid", 1, 8, 6, 4, 3, 3, 7, "VALID"),
        ("c1_same", 3, 5, 5, 16, 1, 1, 125, "SAME"),
        ("c2_same", 1, 6, 7, 8, 2, 2, 33, "SAME"),
        ("c3_wide", 1, 6, 6, 64, 3, 3, 40, "SAME"),
    ]
    for name, B, H, W, C, kh, kw, od, pad in conv_cases:
        x = f32(B, H, W, C)
        k = f32(kh, kw, C, od, lo=-0.5, hi=0.5)
        node = ref.Conv2D("c", _Fake(x), k, [1, 1, 1, 1], pad)
        node.run()
        cases[f"conv_{name}_x"] = x
        cases[f"conv_{name}_k"] = k
        cases[f"conv_{name}_pad"] = np.array(pad)
        cases[f"conv_{name}_y"] = np.asarray(node.result, dtype=np.float32)

    for name, shape in [("a", (2, 5, 7, 16)), ("b", (1, 3, 3, 125)), ("c", (3, 4, 4, 13))]:
        x = f32(*shape, lo=-3, hi=3)
        C = shape[-1]
        b = f32(C)
        node = ref.BiasAdd("b", _Fake(x), b); node.run()
        cases[f"bias_{name}_x"] = x; cases[f"bias_{name}_b"] = b
        cases[f"bias_{name}_y"] = np.asarray(node.result, dtype=np.float32)
        mean = f32(C, lo=-0.2, hi=0.2)
        var = f32(C, lo=0.5, hi=1.5)
        gamma = f32(C, lo=0.5, hi=1.5)
        node = ref.BatchNorm("bn", _Fake(x), mean, var, gamma, 1e-5); node.run()
        cases[f"bn_{name}_x"] = x; cases[f"bn_{name}_mean"] = mean
        cases[f"bn_{name}_var"] = var; cases[f"bn_{name}_gamma"] = gamma
        cases[f"bn_{name}_y"] = np.asarray(node.result, dtype=np.float32)
        node = ref.LeakyReLU("l", _Fake(x)); node.run()
        cases[f"leaky_{name}_x"] = x
        cases[f"leaky_{name}_y"] = np.asarray(node.result, dtype=np.float32)

    pool_cases = [
        ("k2s2_even", (2, 8, 6, 16), (2, 2), (2, 2), "SAME"),
        ("k2s2_odd", (1, 7, 5, 8), (2, 2), (2, 2), "SAME"),
        ("k2s1_same", (1, 13, 13, 32), (2, 2), (1, 1), "SAME"),
        ("k3s2_valid", (2, 9, 9, 4), (3, 3), (2, 2), "VALID"),
        ("k3s2_same", (1, 10, 7, 12), (3, 3), (2, 2), "SAME"),
    ]
    for name, shape, k, s, pad in pool_cases:
        x = f32(*shape, lo=-5, hi=5)
        node = ref.MaxPool2D("p", _Fake(x), [1, k[0], k[1], 1], [1, s[0], s[1], 1], pad)
        node.run()
        cases[f"pool_{name}_x"] = x
        cases[f"pool_{name}_k"] = np.array(k)
        cases[f"pool_{name}_s"] = np.array(s)
        cases[f"pool_{name}_pad"] = np.array(pad)
        cases[f"pool_{name}_y"] = np.asarray(node.result, dtype=np.float32)
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--skip-net", action="store_true")
    args = ap.parse_args()

    ref = load_reference_numpy_engine()
    t0 = time.time()
    cases = op_cases(ref)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **cases)
    print(f"ops.npz: {len(cases)} arrays ({time.time() - t0:.1f}s)", flush=True)

    ws = synth.yolo_weights()
    spec = {
        "generator": synth.__doc__.strip(),
        "channels": list(synth.CHANNELS),
        "in_shape": list(synth.IN_SHAPE),
        "weight_seed": synth.WEIGHT_SEED,
        "weights_sha256": synth.weights_digest(ws),
        "frames": {},
        "reference": "cs492-projects/proj3/dnn.py (numpy/scipy engine), one fresh graph per frame",
        "tolerance": "max|d| <= 1e-4 * max|ref| per tensor (normwise), SURVEY.md §8a",
    }
    if not args.skip_net:
        for i in range(args.frames):
            x = synth.frame(i)
            spec["frames"][str(i)] = hashlib.sha256(x.tobytes()).hexdigest()
            g, nodes = build_yolo(ref, ws, [1, 416, 416, 3])
            t0 = time.time()
            eng = ref.DnnInferenceEngine(g, False)
            y = np.asarray(eng.run(x), dtype=np.float32)
            dt = time.time() - t0
            np.save(os.path.join(HERE, f"net_frame{i}.npy"), y)
            print(f"frame {i}: {dt:.1f}s  out {y.shape} max|y|={np.abs(y).max():.4f}", flush=True)
            if i == 0:
                np.savez_compressed(os.path.join(HERE, "nodes_frame0.npz"), **node_stats(nodes))
                spec["ref_seconds_per_frame"] = round(dt, 2)
    with open(os.path.join(HERE, "spec.json"), "w") as f:
        json.dump(spec, f, indent=1)


if __name__ == "__main__":
    main()
