"""TEST INFRASTRUCTURE ONLY — decision-margin filter for comparing the detections of two
prediction tensors that differ by a bounded perturbation (the fp16 path, BASELINE config 5,
against the fp32 reference output), on top of the postprocessing restatement post_numpy.py
(cs492-projects/proj3/yolov2tiny.py:94-234).

A box (row, col, anchor) is decision-stable under an absolute input margin e when, for EVERY
input within e of the given one:
  * its best class is the same (top logit ahead of the runner-up by more than 2e),
  * its threshold decision `conf * p(best) > 0.3` is the same (interval of the score),
  * each truncated corner int(c -/+ size/2) is the same (interval of the corner);
and two stable candidates whose score intervals overlap must not suppress each other
(IoU > 0.3), since their sort order could flip.  Unstable boxes are dropped from BOTH
tensors (objectness set to -80: a score of ~1e-35, never a candidate), after which the two detection lists
must be identical as multisets (near-tied scores of non-overlapping boxes may reorder).
"""
import numpy as np

import post_numpy as PN

_F = np.float32


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def _box_intervals(p, e):
    """Per box (13,13,5): (stable_class, score_lo, score_hi, corners_lo[4], corners_hi[4]) in
    float64.  e: absolute input margin, a scalar or one value per input [13,13,5,25]."""
    p = np.asarray(p, np.float64).reshape(13, 13, 5, 25)
    e = np.broadcast_to(np.asarray(e, np.float64), (13, 13, 5, 25)).reshape(13, 13, 5, 25)
    tx, ty, tw, th, tc = (p[..., k] for k in range(5))
    ex, ey, ew, eh, ec = (e[..., k] for k in range(5))
    lg = p[..., 5:]
    el = e[..., 5:].max(-1)  # one margin for all class logits of a box
    srt = np.sort(lg, axis=-1)
    best = np.argmax(lg, axis=-1)
    cls_ok = (srt[..., -1] - srt[..., -2]) > 2 * el
    lb = np.take_along_axis(lg, best[..., None], -1)
    rest = np.exp(lg - lb)  # includes the best (=1)
    others = rest.sum(-1) - 1.0
    pb_lo = 1.0 / (1.0 + others * np.exp(2 * el))
    pb_hi = 1.0 / (1.0 + others * np.exp(-2 * el))
    s_lo = _sig(tc - ec) * pb_lo
    s_hi = _sig(tc + ec) * pb_hi
    col = np.arange(13)[None, :, None]
    row = np.arange(13)[:, None, None]
    anc = np.asarray(PN.ANCHORS, np.float64).reshape(5, 2)
    cx_lo, cx_hi = (col + _sig(tx - ex)) * 32, (col + _sig(tx + ex)) * 32
    cy_lo, cy_hi = (row + _sig(ty - ey)) * 32, (row + _sig(ty + ey)) * 32
    w_lo, w_hi = np.exp(tw - ew) * anc[:, 0] * 32, np.exp(tw + ew) * anc[:, 0] * 32
    h_lo, h_hi = np.exp(th - eh) * anc[:, 1] * 32, np.exp(th + eh) * anc[:, 1] * 32
    lo = np.stack([cx_lo - w_hi / 2, cy_lo - h_hi / 2, cx_lo + w_lo / 2, cy_lo + h_lo / 2], -1)
    hi = np.stack([cx_hi - w_lo / 2, cy_hi - h_lo / 2, cx_hi + w_hi / 2, cy_hi + h_hi / 2], -1)
    return cls_ok, s_lo, s_hi, lo, hi


def stable_mask(p, e, pad=1e-3):
    """Boxes whose class, threshold decision and integer corners cannot change within e (the
    corner intervals are widened by `pad` px for the float32 rounding of the reference's own
    arithmetic)."""
    cls_ok, s_lo, s_hi, lo, hi = _box_intervals(p, e)
    thr = float(_F(0.3))
    thr_ok = (s_lo > thr * (1 + 1e-6)) | (s_hi <= thr * (1 - 1e-6))
    corner_ok = np.all(np.trunc(lo - pad) == np.trunc(hi + pad), axis=-1)
    cand = s_lo > thr  # stable candidates (need stable corners); stable non-candidates are fine as is
    return cls_ok & thr_ok & (corner_ok | ~cand), s_lo, s_hi


def drop_unstable(p32, p16, e):
    """Copies of both tensors with every box that is unstable in EITHER tensor removed
    (objectness -80), iterating the overlapping-near-tie rule to a fixed point.  Returns
    (q32, q16, n_stable_candidates)."""
    q32 = np.array(p32, np.float32).reshape(13, 13, 5, 25)
    q16 = np.array(p16, np.float32).reshape(13, 13, 5, 25)
    m32, lo32, hi32 = stable_mask(q32, e)
    m16, lo16, hi16 = stable_mask(q16, e)
    keep = m32 & m16
    thr = float(_F(0.3))
    while True:
        idx = [tuple(i) for i in np.argwhere(keep & (lo32 > thr))]
        boxes = {}
        for i in idx:
            d = PN.decode_one(q32, *i)
            boxes[i] = d
        bad = set()
        for a in range(len(idx)):
            for b in range(a + 1, len(idx)):
                ia, ib = idx[a], idx[b]
                sa = (min(lo32[ia], lo16[ia]), max(hi32[ia], hi16[ia]))
                sb = (min(lo32[ib], lo16[ib]), max(hi32[ib], hi16[ib]))
                if sa[0] <= sb[1] and sb[0] <= sa[1] and PN.iou(boxes[ia][0], boxes[ib][0]) > 0.3:
                    bad.update((ia, ib))
        if not bad:
            break
        for i in bad:
            keep[i] = False
    for q in (q32, q16):
        q[..., 4][~keep] = -80.0
    return q32, q16, len(idx)


def match_rate(d_a, d_b, min_iou=0.9):
    """Fraction of detections [(class, l, t, r, b, score)] of d_a that have a detection of the
    same class with IoU >= min_iou in d_b."""
    if not d_a:
        return 1.0
    hit = 0
    for a in d_a:
        if any(b[0] == a[0] and PN.iou(a[1:5], b[1:5]) >= min_iou for b in d_b):
            hit += 1
    return hit / len(d_a)
