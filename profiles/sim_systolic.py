"""CPU model of the systolic list scan (k_scan_sys, M = 16) used to check the design
before it ran on the GPU: the skewed code image, the 16-row partition and the
completion masks must yield every code of a list exactly once, summed in the
oracle's order (dis0 + tab[0][c0] + ... + tab[15][c15]).

Run: python3 profiles/sim_systolic.py   (design check; the GPU parity tests are the real gate)
"""
import numpy as np


def skew_image(codes):
    """codes [n][16] u8 -> chunks [ceil(n/16) + 1][16 lanes][16 bytes], as upload_lists builds it."""
    n = codes.shape[0]
    nb = (n + 15) // 16 + 1
    img = np.zeros((nb, 16, 16), np.uint8)
    for b in range(nb):
        for m in range(16):
            for t in range(16):
                c = 16 * b + t - m
                if 0 <= c < n:
                    img[b, m, t] = codes[c, m]
    return img


def scan(codes, lut, d0):
    """All 16 rows (4 waves x 4 rows) of one work item, one query; returns {code: distance}."""
    n = codes.shape[0]
    img = skew_image(codes)
    nc = (n + 15) // 16
    lut0 = (np.float32(d0) + lut[0]).astype(np.float32)  # dis0 folded into the m = 0 entries
    out = {}
    for wave in range(4):
        ds = [((nc * (x + 1)) >> 4) - ((nc * x) >> 4) for x in range(wave * 4, wave * 4 + 4)]
        dmin, dmax = min(ds), max(ds)
        for rid in range(wave * 4, wave * 4 + 4):
            rb0, rb1 = (nc * rid) >> 4, (nc * (rid + 1)) >> 4
            cend = min(rb1 * 16, n)
            P = np.full(16, np.nan, np.float32)
            for i in range(dmax + 1):
                chunk = img[min(rb0 + i, nc)]
                cb = 16 * (rb0 + i) - 15
                for t in range(16):
                    prev = np.concatenate([[np.float32(0)], P[:15]])  # row_shr:1, lane 0 reads 0
                    vals = np.array([lut0[chunk[0, t]]] + [lut[m, chunk[m, t]] for m in range(1, 16)], np.float32)
                    P = (prev + vals).astype(np.float32)
                    code = cb + t
                    ok = not np.isnan(P[15]) and (i < dmin or code < cend)
                    if ok:
                        assert code not in out, f"code {code} completed twice"
                        assert 0 <= code < n, code
                        out[code] = P[15]
    return out


def oracle(codes, lut, d0):
    res = np.empty(codes.shape[0], np.float32)
    for c in range(codes.shape[0]):
        dis = np.float32(d0)
        for m in range(16):
            dis = np.float32(dis + lut[m, codes[c, m]])
        res[c] = dis
    return res


def main():
    rng = np.random.default_rng(0)
    for n in (1, 2, 15, 16, 17, 31, 33, 100, 255, 256, 257, 977, 1774):
        codes = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        lut = (rng.normal(size=(16, 256)) * 10).astype(np.float32)
        d0 = np.float32(rng.normal() * 100)
        got = scan(codes, lut, d0)
        assert sorted(got) == list(range(n)), (n, len(got))
        g = np.array([got[c] for c in range(n)], np.float32)
        assert np.array_equal(g, oracle(codes, lut, d0)), n
        print(f"n={n}: every code once, bit-identical to the sequential sum")


if __name__ == "__main__":
    main()
