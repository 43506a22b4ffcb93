"""TEST INFRASTRUCTURE ONLY — numpy restatement of the frame preprocessing of the
reference driver (cs492-projects/proj3/__init__.py:8-12: cv2.resize(im, (416, 416)) /
255., BGR -> RGB, float32), with cv2.resize's INTER_LINEAR for 8-bit images written out as
OpenCV's scalar fixed-point algorithm (11-bit coefficients, rounding shift of 22 bits).
cv2 is not importable in this image, so the resize half is PARITY UNPINNED (checked only
against this restatement and against the exact identity-size case); used by tests/ only.
"""
import numpy as np


def _axis(dst, src):
    scale = src / dst
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo], f[lo] = 0, np.float32(0)
    hi = s >= src - 1
    s[hi], f[hi] = src - 1, np.float32(0)
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    s1 = np.minimum(s + 1, src - 1)
    return s, s1, a0, a1


def resize_linear_u8(im, oh, ow):
    im = np.asarray(im, dtype=np.uint8)
    h, w = im.shape[:2]
    if (h, w) == (oh, ow):
        return im.copy()
    xs0, xs1, xa0, xa1 = _axis(ow, w)
    ys0, ys1, ya0, ya1 = _axis(oh, h)
    I = im.astype(np.int64)
    r0 = xa0[None, :, None] * I[ys0][:, xs0] + xa1[None, :, None] * I[ys0][:, xs1]
    r1 = xa0[None, :, None] * I[ys1][:, xs0] + xa1[None, :, None] * I[ys1][:, xs1]
    o = (ya0[:, None, None] * r0 + ya1[:, None, None] * r1 + (1 << 21)) >> 22
    return np.clip(o, 0, 255).astype(np.uint8)


def resize_input(im, size=416):
    """__init__.py:8-12 with the restated resize."""
    imsz = resize_linear_u8(im, size, size)
    imsz = imsz / 255.
    imsz = imsz[:, :, ::-1]
    return np.asarray(imsz, dtype=np.float32)
