"""emu_v10.py — numpy emulation of the radix-16 forward transform of the v10 blind rotation,
lane by lane, before any HIP: the two digit polynomials of one accumulator polynomial split over
the wave's halves, a radix-16 register pass, ONE LDS transpose (slot map checked for bank
conflicts), a second radix-16 register pass, the last radix-2 stage across lanes 16 apart
(v_permlane16_swap), and the re-pairing of both digits' spectra in every lane (v_permlane32_swap),
which leaves slot 8 L' + r of layout C in lane L with L' = (L >> 5) + 2 ((L >> 4) & 1) + 4 (L & 15).
Checked against emu_v6's forward (the same merged-twist transform) on every position.

    python scripts/emu_v10.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import emu_v6 as E  # noqa: E402

W, _ = E.twiddles_v6()


def cis(e):
    return E.cis(e)


def bf(x, r0, r1, tw):
    """x [lanes][regs]; tw broadcastable [lanes]"""
    t = tw * x[:, r1]
    x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t


def permlane32_swap(a, b):
    """v_permlane32_swap vdst=a, src=b: a's lanes 32-63 <-> b's lanes 0-31 (per register)"""
    a, b = a.copy(), b.copy()
    a[32:], b[:32] = b[:32].copy(), a[32:].copy()
    return a, b


def permlane16_swap(a, b):
    """v_permlane16_swap vdst=a, src=b: a's odd rows (lanes 16-31, 48-63) <-> b's even rows
    (lanes 0-15, 32-47)"""
    a, b = a.copy(), b.copy()
    for lo, hi in ((0, 16), (32, 48)):
        a[hi:hi + 16], b[lo:lo + 16] = b[lo:lo + 16].copy(), a[hi:hi + 16].copy()
    return a, b


HALF = 528   # slots per half (digit polynomial): 512 positions + 16 pad


def slot(n):
    """LDS slot of position n within a half's region: n + (n >> 5), linear in the register index
    on both sides (immediate offsets: store l + 33 r', load b' + 33 m + 2 r'')"""
    return n + (n >> 5)


def bank_conflicts(slots_by_lane):
    """16-B accesses: a wave's 64 lanes in 4 groups of 16 (256 B / clock); conflict-free when the
    16 slots of a group are distinct mod 16 (each slot covers 4 of the 64 four-byte banks)"""
    worst = 1
    for g in range(4):
        s = np.asarray(slots_by_lane[16 * g:16 * g + 16]) % 16
        worst = max(worst, int(np.max(np.bincount(s, minlength=16))))
    return worst


def forward_v10(hi, lo):
    """hi, lo: the two digit polynomials (1024 each) of one accumulator polynomial.  Returns
    D [64 lanes][2 digits][8 regs] with D[L][d][r] = spectrum of digit d at position 8 L' + r."""
    L = np.arange(64)
    l = L & 31
    # acc layout A: lane L holds coefficients L + 64 r (r < 16); HI / LO = the digits there
    HI = np.stack([hi[L + 64 * r] for r in range(16)], axis=1).astype(complex)
    LO = np.stack([lo[L + 64 * r] for r in range(16)], axis=1).astype(complex)
    # digit exchange: swap(vdst = HI[r], src = LO[r]): lower lanes end with hi digits of
    # coefficients l + 64 r (HI) and l + 32 + 64 r (LO); upper lanes with lo digits of both
    for r in range(16):
        HI[:, r], LO[:, r] = permlane32_swap(HI[:, r], LO[:, r])
    Ev, Od = HI, LO
    # fold: position n = l + 32 r' -> Z[r'] = a_n + i a_{n + 512}
    Z = np.empty((64, 16), dtype=complex)
    for k in range(8):
        Z[:, 2 * k] = Ev[:, k] + 1j * Ev[:, k + 8]
        Z[:, 2 * k + 1] = Od[:, k] + 1j * Od[:, k + 8]
    # pass 1: stages 0..3 (bits 8..5 of n = bits 3..0 of r'), uniform twiddles
    for k in range(4):
        dist = 8 >> k
        for r in range(16):
            if r & dist:
                continue
            b = r >> (4 - k)          # block of stage k
            bf(Z, r, r + dist, cis(W[k][b]))
    # transpose through LDS: half h region h * 512; source lane l reg r' holds n = l + 32 r'
    lds = np.full(2 * HALF, np.nan, dtype=complex)
    for r in range(16):
        n = l + 32 * r
        s = slot(n) + HALF * (L >> 5)
        assert bank_conflicts(s) == 1, ("store", r)
        lds[s] = Z[:, r]
    m, bb = L & 15, (L >> 4) & 1
    X = np.empty((64, 16), dtype=complex)
    for r in range(16):             # target lane (m, b') reg r'' holds n = b' + 2 r'' + 32 m
        n = bb + 2 * r + 32 * m
        s = slot(n) + HALF * (L >> 5)
        assert bank_conflicts(s) == 1, ("load", r)
        X[:, r] = lds[s]
    # pass 2: stages 4..7 on bits 4..1 of n = bits 3..0 of r''; per-lane twiddles
    tw4 = cis(np.array([W[4][mm] for mm in m]))                        # block m (either parity)
    for r in range(8):
        bf(X, r, r + 8, tw4)
    t5 = cis(np.array([W[5][2 * mm] for mm in m]))
    for r in range(16):
        if r & 4:
            continue
        odd = r >> 3                                                   # block 2m + (r >> 3)
        bf(X, r, r + 4, t5 * (1j if odd else 1))
    t6 = [cis(np.array([W[6][4 * mm + 2 * q] for mm in m])) for q in range(2)]
    for r in range(16):
        if r & 2:
            continue
        blk = r >> 2                                                   # block 4m + (r >> 2)
        bf(X, r, r + 2, t6[blk >> 1] * (1j if blk & 1 else 1))
    t7 = [cis(np.array([W[7][8 * mm + 2 * q] for mm in m])) for q in range(4)]
    for r in range(0, 16, 2):
        blk = r >> 1                                                   # block 8m + (r >> 1)
        bf(X, r, r + 1, t7[blk >> 1] * (1j if blk & 1 else 1))
    # stage 8 (bit 0 = lane bit 4): swap(vdst = x[p], src = x[p + 8]) -> lane (m, b') pair p holds
    # positions n0 = 2 p + 16 b' + 32 m (x[p]) and n0 + 1 (x[p + 8])
    for p in range(8):
        X[:, p], X[:, p + 8] = permlane16_swap(X[:, p], X[:, p + 8])
    t8 = [cis(np.array([W[8][16 * mm + 8 * b_ + 2 * q] for mm, b_ in zip(m, bb)])) for q in range(4)]
    for p in range(8):
        bf(X, p, p + 8, t8[p >> 1] * (1j if p & 1 else 1))
    # now reg q = p + 8 e holds position 2 p + e + 16 b' + 32 m.  Re-pair: for p in 0..3 swap
    # (vdst = reg p + 8e [bit 3 = 0], src = reg p + 4 + 8e [bit 3 = 1]): lower lanes keep digit
    # hi at bit 3 = 0 and receive digit lo's bit-3 = 0 value; upper lanes the bit-3 = 1 pair
    for e in range(2):
        for p in range(4):
            q0, q1 = p + 8 * e, p + 4 + 8 * e
            X[:, q0], X[:, q1] = permlane32_swap(X[:, q0], X[:, q1])
    D = np.empty((64, 2, 8), dtype=complex)
    for e in range(2):
        for p in range(4):
            r = e + 2 * p                                               # bits 0..2 of n
            D[:, 0, r] = X[:, p + 8 * e]
            D[:, 1, r] = X[:, p + 4 + 8 * e]
    return D


def inverse_c16_slot(n):
    """the inverse's C -> B transpose from this lane order (fft_wave.h store_C16 / load_B16):
    position n at 16 (n >> 3) + ((n & 7) ^ t((n >> 3) >> 2)), t = bits 1 and 3 exchanged"""
    k, j = n >> 3, n & 7
    m = k >> 2
    t = (m & 5) | ((m >> 2) & 2) | ((m & 2) << 2)
    return 16 * k + (j ^ t)


def check_inverse_c16():
    L = np.arange(64)
    Lp = logical_lane(L)
    s = [inverse_c16_slot(n) for n in range(512)]
    assert len(set(s)) == 512 and max(s) < 1024
    for r in range(8):
        assert bank_conflicts([inverse_c16_slot(8 * lp + r) for lp in Lp]) == 1, ("store C16", r)
        assert bank_conflicts([inverse_c16_slot((l & 7) + 8 * r + 64 * (l >> 3)) for l in L]) == 1, ("load B16", r)


def logical_lane(L):
    return (L >> 5) + 2 * ((L >> 4) & 1) + 4 * (L & 15)


def main():
    T = E.tables()
    rng = np.random.default_rng(10)
    hi = rng.integers(-512, 512, 1024)
    lo = rng.integers(-512, 512, 1024)
    D = forward_v10(hi, lo)
    L = np.arange(64)
    Lp = logical_lane(L)
    assert sorted(Lp) == list(range(64))
    worst = 0.0
    for d, poly in enumerate((hi, lo)):
        ref = np.empty(512, dtype=complex)
        ref[E.IDX_C] = E.fwd(poly.astype(float), T)          # position n = slot 8 L + r
        for r in range(8):
            got = D[:, d, r]
            want = ref[8 * Lp + r]
            worst = max(worst, float(np.max(np.abs(got - want))))
    assert worst < 1e-6, worst
    check_inverse_c16()
    print(f"emu_v10: radix-16 forward == emu_v6 forward on every position (max |diff| {worst:.2e}); "
          "LDS transposes (forward, inverse C16) conflict-free; lane map L' = (L>>5) + 2((L>>4)&1) + 4(L&15)")


if __name__ == "__main__":
    main()
