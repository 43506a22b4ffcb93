"""Bank-conflict model of the x3 patch kernels' A-fragment reads (ds_read_b128), per LDS row
layout, for YOLOv2-tiny conv6/conv7 at batch 64 (13x13 frames, 176-row tiles, 9 taps, 3 bf16
pieces).  Extra LDS cycles per ds_read_b128 = sum over its four 16-lane groups of (the largest
number of lanes on one 16-byte bank quad - 1) (MI355X_MICROARCH.md section LDS).  The model
reproduces the counters: 192-B rows 7.1 (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS measured 6.8),
the round-2 XOR swizzle 4.0 (measured 3.5).

  python tools/lds_conflict_model.py
"""
# ds_read_b128 lane groups: {0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same + 32
G = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
     list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G += [[lane + 32 for lane in g] for g in G]
H = W = 13
WP = W + 2
BM = 176
B = 64
M = B * H * W


def padded(m):
    b, r = divmod(m, H * W)
    oy, ox = divmod(r, W)
    return (b * (H + 2) + oy + 1) * WP + ox + 1


def extra_cycles(pitch_units, slot, tiles=range(0, 62)):
    """mean extra LDS cycles per fragment read; row r's (piece p, k slot fq) 16-B unit sits at
    pitch_units * r + slot(r, p, fq)"""
    tot = n = 0
    for tm in tiles:
        m0 = tm * BM
        p0 = padded(m0) - (WP + 1)
        for i in range(BM // 16):
            rows = [padded(min(m0 + 16 * i + fr, M - 1)) - p0 for fr in range(16)]
            for t in range(9):
                toff = (t // 3 - 1) * WP + (t % 3 - 1)
                for p in range(3):
                    for g in G:
                        cnt = {}
                        for lane in g:
                            r = rows[lane & 15] + toff
                            u = (pitch_units * r + slot(r, p, lane >> 4)) % 16
                            cnt[u] = cnt.get(u, 0) + 1
                        tot += max(cnt.values()) - 1
                    n += 1
    return tot / n


def main():
    plain = lambda r, p, fq: 4 * p + fq  # noqa: E731
    swizzled = lambda r, p, fq: 4 * p + (fq ^ ((r >> 1) & 2))  # noqa: E731  (round-2 kernel)
    print("192-B rows, plain            %.2f" % extra_cycles(12, plain))
    print("192-B rows, XOR swizzle      %.2f" % extra_cycles(12, swizzled))
    for units in (13, 14, 15, 16, 18):
        print("%d-B rows, plain            %.2f" % (16 * units, extra_cycles(units, plain)))


if __name__ == "__main__":
    main()
