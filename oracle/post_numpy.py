"""TEST INFRASTRUCTURE ONLY — restatement of the reference's YOLOv2 postprocessing
(cs492-projects/proj3/yolov2tiny.py:94-234: decode, 0.3 score threshold, stable sort, greedy
NMS) with the exact numeric semantics the reference has under this image's numpy 2.2:

  * every scalar op on the np.float32 predictions stays float32 (Python scalars are "weak",
    NEP 50): sigmoid = 1 / (1 + float32(e) ** -x)            (yolov2tiny.py:229-230)
    centre = (col + sigmoid(t)) * 32, size = exp(t) * anchor * 32   (:122-127)
  * softmax: exp(x - max(x)) / sum, the sum in numpy's float32 pairwise order (8 partial
    sums for a 20-vector, then the tail)                      (:232-234)
  * best class = first index of the max                        (:132-134)
  * corners = int(float32 centre -/+ float32 size / 2), truncation toward zero, for EVERY
    box before thresholding (so a non-finite corner raises, as in the reference)  (:137-140)
  * keep if float32(conf * class score) > float32(0.3)         (:142)
  * stable descending sort by score (Python list.sort)         (:146)
  * greedy NMS: drop a box if its IoU with ANY already kept box is > 0.3, IoU on the integer
    corners with +1 widths and NO clamp of negative overlaps, exact Python ints, then
    int / float(int) in float64                                (:179-221)

Used by tests/ (checker, pinned by tests/golden/post_*, generated from the reference's own
functions by tests/golden/make_golden_post.py) and nowhere in the product path.
"""
import numpy as np

N_CLASSES = 20
ANCHORS = (1.08, 1.19, 3.42, 4.41, 6.63, 11.38, 9.42, 5.11, 16.62, 10.52)  # yolov2tiny.py:110
CLASSES = ("aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair", "cow", "diningtable",
           "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa", "train", "tvmonitor")
COLORS = ((254.0, 254.0, 254), (239.88888888888889, 211.66666666666669, 127),
          (225.77777777777777, 169.33333333333334, 0), (211.66666666666669, 127.0, 254),
          (197.55555555555557, 84.66666666666667, 127), (183.44444444444443, 42.33333333333332, 0),
          (169.33333333333334, 0.0, 254), (155.22222222222223, -42.33333333333335, 127),
          (141.11111111111111, -84.66666666666664, 0), (127.0, 254.0, 254),
          (112.88888888888889, 211.66666666666669, 127), (98.77777777777777, 169.33333333333334, 0),
          (84.66666666666667, 127.0, 254), (70.55555555555556, 84.66666666666667, 127),
          (56.44444444444444, 42.33333333333332, 0), (42.33333333333332, 0.0, 254),
          (28.222222222222236, -42.33333333333335, 127), (14.111111111111118, -84.66666666666664, 0),
          (0.0, 254.0, 254), (-14.111111111111118, 211.66666666666669, 127))

_F = np.float32
_E = _F(np.e)
_THR = _F(0.3)


def _pairwise_sum_f32(a):
    """numpy's float32 add.reduce order for a contiguous vector of <= 128 elements."""
    n = len(a)
    if n < 8:
        r = _F(0)
        for v in a:
            r = _F(r + v)
        return r
    r = [a[j] for j in range(8)]
    i = 8
    while i < n - (n % 8):
        for j in range(8):
            r[j] = _F(r[j] + a[i + j])
        i += 8
    res = _F(_F(_F(r[0] + r[1]) + _F(r[2] + r[3])) + _F(_F(r[4] + r[5]) + _F(r[6] + r[7])))
    while i < n:
        res = _F(res + a[i])
        i += 1
    return res


def _sigmoid(x):
    return _F(_F(1) / _F(_F(1) + _E ** _F(-x)))


def decode_one(p, row, col, b):
    """Box (row, col, anchor) of a [13,13,5,25] float32 tensor: [[left, top, right, bottom],
    score, class] (yolov2tiny.py:118-140)."""
    tx, ty, tw, th, tc = (p[row, col, b, k] for k in range(5))
    cx = _F(_F(_F(col) + _sigmoid(tx)) * _F(32.0))
    cy = _F(_F(_F(row) + _sigmoid(ty)) * _F(32.0))
    rw = _F(_F(np.exp(tw) * _F(ANCHORS[2 * b])) * _F(32.0))
    rh = _F(_F(np.exp(th) * _F(ANCHORS[2 * b + 1])) * _F(32.0))
    conf = _sigmoid(tc)
    logits = p[row, col, b, 5:]
    e = np.exp(logits - np.max(logits))
    s = _pairwise_sum_f32(e)
    probs = [_F(v / s) for v in e]
    best = max(range(N_CLASSES), key=lambda k: (probs[k], -k))
    left = int(_F(cx - _F(rw / _F(2.0))))
    right = int(_F(cx + _F(rw / _F(2.0))))
    top = int(_F(cy - _F(rh / _F(2.0))))
    bottom = int(_F(cy + _F(rh / _F(2.0))))
    return [[left, top, right, bottom], _F(conf * probs[best]), best]


def decode(predictions):
    """All 845 boxes of one image in (row, col, anchor) order:
    [(left, top, right, bottom), score, class] for those above the threshold (unsorted)."""
    p = np.asarray(predictions, dtype=np.float32).reshape(13, 13, 5, 25)
    out = []
    for row in range(13):
        for col in range(13):
            for b in range(5):
                d = decode_one(p, row, col, b)
                if d[1] > _THR:
                    out.append(d)
    return out


def iou(a, b):
    xa, ya, xb, yb = max(a[0], b[0]), max(a[1], b[1]), min(a[2], b[2]), min(a[3], b[3])
    inter = (xb - xa + 1) * (yb - ya + 1)
    area_a = (a[2] - a[0] + 1) * (a[3] - a[1] + 1)
    area_b = (b[2] - b[0] + 1) * (b[3] - b[1] + 1)
    return inter / float(area_a + area_b - inter)


def detect(predictions):
    """Post-NMS detections [(class, left, top, right, bottom, score)] in output order."""
    cand = decode(predictions)
    cand.sort(key=lambda t: t[1], reverse=True)
    kept = []
    for c in cand:
        # every kept box is tested, no early exit (yolov2tiny.py:209-216): a zero IoU
        # denominator anywhere in the list raises, as in the reference
        hits = [iou(c[0], k[0]) > 0.3 for k in kept]
        if not any(hits):
            kept.append(c)
    return [(k[2], k[0][0], k[0][1], k[0][2], k[0][3], float(k[1])) for k in kept]


def postprocessing(predictions):
    """Same return value as yolov2tiny.postprocessing: [(name, (l, t), (r, b), color)]."""
    return [(CLASSES[c], (l, t), (r, b), COLORS[c]) for c, l, t, r, b, _ in detect(predictions)]


def synthetic_predictions(rng, n_hot=None, tw_scale=1.0):
    """A [13,13,125] prediction tensor with many boxes above the threshold: objectness and one
    class logit per box boosted so conf * p(class) crosses 0.3 for a good fraction."""
    p = rng.standard_normal((13, 13, 5, 25)).astype(np.float32)
    p[..., 2:4] *= np.float32(tw_scale)
    p[..., 4] = (rng.standard_normal((13, 13, 5)) * 3.0).astype(np.float32)
    hot = rng.integers(0, 20, size=(13, 13, 5))
    boost = rng.uniform(0.0, 8.0, size=(13, 13, 5)).astype(np.float32)
    np.put_along_axis(p[..., 5:], hot[..., None], (np.take_along_axis(p[..., 5:], hot[..., None], -1)
                                                     + boost[..., None]).astype(np.float32), -1)
    if n_hot is not None:  # keep only n_hot random boxes above threshold
        keep = rng.permutation(845)[:n_hot]
        mask = np.zeros(845, bool)
        mask[keep] = True
        p.reshape(845, 25)[~mask, 4] = -20.0
    return p.reshape(13, 13, 125)
