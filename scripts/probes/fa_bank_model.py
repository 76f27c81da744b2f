"""LDS bank-conflict model of the flash-attention dK/dV kernel's reads (gfx950 lane groups from
MI355X_MICROARCH.md 'LDS': ds_read_b128 = 4 x 16-lane groups, ds_read_b64_tr_b16 = 2 x 32).

Counts LDS-array cycles per wave-instruction for the two access patterns of bwd_dkdv_kernel over
a swizzled [64][128] 16-bit image (256-byte rows, 16-byte chunks XOR-swizzled by swz(row)):
  row reads   row nt*16 + (lane & 15), chunk 4ks + (lane >> 4)                  (S, dP operands)
  tr reads    rows 32ks + 4g + (L >> 2) and 32ks + 16 + 4g + (L >> 2), col 16n + 4(L & 3)
Usage: python scripts/probes/fa_bank_model.py [--search]   (--search: all 4x4 linear swizzles)
"""
import sys

B128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
B128 = B128 + [[l + 32 for l in g] for g in B128]
TR64 = [list(range(32)), list(range(32, 64))]


def cycles(addrs, groups, ndw):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            for d in range(ndw):
                w = addrs[l] // 4 + d
                banks.setdefault(w % 64, set()).add(w)
        tot += max(len(s) for s in banks.values())
    return tot


def score(swz):
    def off(row, ch):
        return row * 256 + ((ch ^ swz(row)) << 4)
    rr = sum(cycles([off(nt * 16 + (l & 15), 4 * ks + (l >> 4)) for l in range(64)], B128, 4)
             for nt in range(4) for ks in range(4))
    tr = 0
    for ks in range(2):
        for n in range(8):
            for hi in range(2):
                addrs = []
                for l in range(64):
                    L, g = l & 15, l >> 4
                    col = 16 * n + 4 * (L & 3)
                    r = 32 * ks + 16 * hi + 4 * g + (L >> 2)
                    addrs.append(off(r, col >> 3) + 8 * ((col >> 2) & 1))
                tr += cycles(addrs, TR64, 2)
    return rr, tr   # ideal: 64 (16 b128 reads x 4 groups), 64 (32 tr reads x 2 groups)


def linear(cols):
    def swz(r):
        v = 0
        for i in range(4):
            if (r >> i) & 1:
                v ^= cols[i]
        return v
    return swz


if __name__ == "__main__":
    print("default swz (fwd/dq images):", score(lambda r: ((r & 3) << 2) | ((r >> 2) & 3)))
    print("SW=1 (dK/dV images)        :", score(linear([8, 4, 2, 0])))
    if "--search" in sys.argv:   # ~10 min in CPython
        ok = [m for m in range(1 << 16)
              if score(linear([(m >> (4 * i)) & 15 for i in range(4)])) == (64, 64)]
        print(len(ok), "conflict-free linear swizzles")
