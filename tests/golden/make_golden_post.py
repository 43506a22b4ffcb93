"""Generate the postprocessing fixtures under tests/golden/ from the REFERENCE's own
functions (build container only; /root/reference never exists on the GPU box):

    python tests/golden/make_golden_post.py

`cs492-projects/proj3/yolov2tiny.py` imports dnn_openblas, which loads its C library at
import time, so the module itself is not importable here.  Its postprocessing functions
(postprocessing, iou, non_maximal_suppression, sigmoid, softmax; yolov2tiny.py:94-234) are
self-contained: this script parses the file, compiles only those function definitions with
numpy in scope and calls them.  Nothing of the reference is copied into the repository.

Writes  post_cases.npz   inputs: [N,13,13,125] fp32 synthetic prediction tensors (the
                         net_frame cases read the committed net_frame*.npy)
        post_golden.json expected outputs: per case the reference's label_boxes
                         [class name, [left, top], [right, bottom]], or
                         {"raises": "ZeroDivisionError"} where the reference raises
Cases: the 4 whole-net golden outputs (net_frame*.npy) and seeded synthetic tensors from
oracle/post_numpy.synthetic_predictions (many candidates, ties, large boxes, empty).
"""
import ast
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import post_numpy  # noqa: E402

REF = "/root/reference/cs492-projects/proj3/yolov2tiny.py"
FUNCS = ("postprocessing", "iou", "non_maximal_suppression", "sigmoid", "softmax")


def load_reference_postprocessing():
    tree = ast.parse(open(REF).read(), REF)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert sorted(d.name for d in defs) == sorted(FUNCS)
    ns = {"np": np}
    exec(compile(ast.Module(body=defs, type_ignores=[]), REF, "exec"), ns)
    return ns["postprocessing"]


def cases():
    out, names = [], []
    for i in range(4):
        out.append(np.load(os.path.join(HERE, f"net_frame{i}.npy")).reshape(13, 13, 125))
        names.append(f"net_frame{i}")
    rng = np.random.default_rng(2024)
    for i in range(3):
        out.append(post_numpy.synthetic_predictions(rng))
        names.append(f"synthetic_dense{i}")
    for n_hot in (0, 1, 7):
        out.append(post_numpy.synthetic_predictions(rng, n_hot=n_hot))
        names.append(f"synthetic_hot{n_hot}")
    # equal scores at different cells: the stable sort keeps (row, col, anchor) order
    p = post_numpy.synthetic_predictions(rng, n_hot=0).reshape(845, 25)
    row = p[0].copy()
    row[4] = 6.0
    row[5:] = -4.0
    row[5 + 11] = 6.0
    for k in (3, 200, 401, 402, 844):
        p[k] = row
    out.append(p.reshape(13, 13, 125))
    names.append("synthetic_ties")
    # big boxes: corner products beyond 64 bits in the IoU
    out.append(post_numpy.synthetic_predictions(rng, tw_scale=9.0))
    names.append("synthetic_big_boxes")
    # an image on which the reference raises ZeroDivisionError: overlaps are not clamped, so
    # area_a + area_b - inter can be 0 for some (candidate, kept) pair
    rng77 = np.random.default_rng(77)
    zd = [post_numpy.synthetic_predictions(rng77, tw_scale=(1.0 if i % 4 else 6.0)) for i in range(5)][4]
    out.append(zd)
    names.append("synthetic_zero_iou_denominator")
    return np.stack(out).astype(np.float32), names


def main():
    ref_post = load_reference_postprocessing()
    preds, names = cases()
    gold = {}
    for name, p in zip(names, preds):
        try:
            boxes = ref_post(p)
        except ZeroDivisionError:
            gold[name] = {"raises": "ZeroDivisionError"}
            print(f"{name:22s} raises ZeroDivisionError")
            continue
        gold[name] = [[b[0], list(b[1]), list(b[2])] for b in boxes]
        print(f"{name:22s} {len(boxes):4d} detections")
    # the net_frame inputs are the committed net_frame*.npy themselves; store only the rest
    syn = [i for i, n in enumerate(names) if not n.startswith("net_frame")]
    np.savez_compressed(os.path.join(HERE, "post_cases.npz"), preds=preds[syn],
                        names=np.array([names[i] for i in syn]))
    with open(os.path.join(HERE, "post_golden.json"), "w") as f:
        json.dump({"source": "cs492-projects/proj3/yolov2tiny.py:94-234 (postprocessing) under numpy "
                             + np.__version__, "cases": gold}, f, indent=0)


if __name__ == "__main__":
    main()
