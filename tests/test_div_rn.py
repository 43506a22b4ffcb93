"""The BN epilogue's division (csrc/gemm_f32.h div_rn): x / d correctly rounded as
RN32(RN64(x * RN64(1/d))).  The header carries the proof (no quotient of two 24-bit
significands lies within 2^-49 relative of a float midpoint; the double product is within
2^-52).  This CPU test restates the same three roundings in numpy and checks them against
IEEE float32 division: every x significand of one binade (the result scales exactly with x's
exponent) for divisors at the edges of the significand range and for the YOLOv2-tiny plan's
real BN divisors sqrtf(var + eps), plus random pairs over the whole normal range.  The GPU
side is covered bit for bit by the element-wise and fused-epilogue GPU tests."""
import numpy as np

import synth


def _div_rn(x, d):
    y = np.float64(1.0) / d.astype(np.float64)
    return (x.astype(np.float64) * y).astype(np.float32)


def _all_significands(lo=1.0):
    bits = np.arange(1 << 23, dtype=np.uint32) | np.uint32(127 << 23)
    return bits.view(np.float32) * np.float32(lo)


def test_div_rn_exhaustive_significands():
    x = _all_significands()
    one = np.float32(1.0)
    edge = [one, np.nextafter(one, np.float32(2)), np.float32(1.5), np.nextafter(np.float32(2), one),
            np.float32(1.3333333), np.float32(1.7320508)]
    ws = synth.yolo_weights()
    plan = [np.sqrt(w["moving_variance"] + np.float32(1e-5)).astype(np.float32) for w in ws if "moving_variance" in w]
    plan = np.concatenate(plan)
    sample = plan[np.random.default_rng(0).choice(len(plan), 10, replace=False)]
    for d in list(edge) + list(sample):
        d = np.float32(d)
        dv = np.full_like(x, d)
        with np.errstate(all="ignore"):
            got, ref = _div_rn(x, dv), x / dv
        bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
        assert bad.size == 0, (float(d), x[bad[:4]])


def test_div_rn_random_pairs_and_plan_divisors():
    rng = np.random.default_rng(1)
    n = 4_000_000
    sig = (rng.integers(0, 1 << 23, n, dtype=np.uint32) | np.uint32(1 << 23)).astype(np.uint32)
    ex = rng.integers(127 - 60, 127 + 60, n).astype(np.uint32)
    x = ((ex << 23) | (sig & np.uint32((1 << 23) - 1)) | (rng.integers(0, 2, n).astype(np.uint32) << 31)).view(np.float32)
    ws = synth.yolo_weights()
    plan = np.concatenate([np.sqrt(w["moving_variance"] + np.float32(1e-5)).astype(np.float32)
                           for w in ws if "moving_variance" in w])
    d = np.where(rng.integers(0, 2, n) == 0, plan[rng.integers(0, len(plan), n)],
                 np.abs(rng.standard_normal(n).astype(np.float32)) + np.float32(1e-3))
    got, ref = _div_rn(x, d), x / d
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
