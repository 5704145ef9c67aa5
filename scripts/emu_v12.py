"""emu_v12.py — numpy emulation of the v12 (four waves per ciphertext) blind-rotation step, layout
by layout, before any HIP: checks that the half-transform data flow computes the exact negacyclic
external product and equals v6's transform slot for slot.  (Round 6: v12 was then built from this,
was Torus32-exact on the GPU first time and measured 2.6 % slower than v6 at B = 1; removed from
the library, DESIGN.md §5.6, profiles/r06_v12_four_wave_latency_priced.txt.)

v12 splits each 512-point transform at its first Cooley-Tukey stage.  Stage 0 of the merged-twist
transform (emu_v6.twiddles_v6) maps z_n, z_{n+256} to u + W0 v (slots 0..255, "half 0") and
u - W0 v (slots 256..511, "half 1"); every later stage stays inside one half.  So wave (w, h) of a
ciphertext:
  * holds the whole accumulator polynomial w (16 Torus32 per lane, the same in both waves of the
    pair) and computes all of its digits (z_n for n = L + 64 r, r < 8: layout A);
  * computes ONLY its half of stage 0 (4 FMAs per output), then stages 1..8 of that half for both
    digit polynomials: 4 complex per lane per polynomial, four radix-4 passes on layouts
        A': m = L + 64 r'              (stages 1, 2: uniform twiddles)
        B': m = (L & 15) + 16 r' + 64 (L >> 4)   (stages 3, 4)
        C': m = (L & 3) + 4 r' + 16 (L >> 2)     (stages 5, 6)
        D': m = 4 L + r'               (stages 7, 8)     slot n = 256 h + m;
  * MACs its half of the slots with the key (v6's key layout: slot n at [r6 = n & 7][L6 = n >> 3])
    for both outputs, hands output 1 - w's partial sum to wave (1 - w, h) (barrier 1);
  * runs the radix-2 DIT inverse stages 0..7 of output w inside its half (layouts D' -> C' -> B'
    -> A', per-lane twiddles e^{-2 pi i j / 2^(k+1)}, j = slot mod 2^k; the post-twist's lane factor
    zeta^-L folded into the inputs of pass A'), stores its half in layout A and loads the partner's
    (barrier 2), and computes stage 8, the register post-twist factors and the rounding for all
    16 coefficients — so both waves of the pair hold the same new accumulator.

    python scripts/emu_v12.py
"""
import numpy as np

import emu_v6 as E

L64 = np.arange(64)
RP = np.arange(4)
# position m (0..255) of lane L, register r' in each half layout
IDX = {
    "A": L64[:, None] + 64 * RP[None, :],
    "B": (L64[:, None] & 15) + 16 * RP[None, :] + 64 * (L64[:, None] >> 4),
    "C": (L64[:, None] & 3) + 4 * RP[None, :] + 16 * (L64[:, None] >> 2),
    "D": 4 * L64[:, None] + RP[None, :],
}


def relayout(x, src, dst):
    flat = np.empty(256, dtype=complex)
    flat[IDX[src]] = x
    return flat[IDX[dst]]


def wt(W, s, b):
    """twiddle of stage s, block b (odd blocks: i x their even sibling, as stored in W)"""
    return E.cis(W[s][b])


def fwd_pass4(x, ta, tb):
    """radix-4 pass on 4 registers: stage a at register distance 2 (twiddle ta), stage b at
    distance 1 (tb for pair (0,1), i tb for pair (2,3)); ta, tb per lane [64]"""
    x = x.copy()

    def bf(r0, r1, tw):
        t = tw * x[:, r1]
        x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t
    bf(0, 2, ta)
    bf(1, 3, ta)
    bf(0, 1, tb)
    bf(2, 3, 1j * tb)
    return x


def fwd_half(zA, h, W):
    """zA [64][8]: the whole folded digit polynomial in layout A (n = L + 64 r).  Returns half h
    of the spectrum in layout D' ([64][4], slot 256 h + 4 L + r')."""
    w0 = wt(W, 0, 0)
    s = 1.0 if h == 0 else -1.0
    x = zA[:, :4] + s * w0 * zA[:, 4:]                              # stage 0, this half only
    one = np.ones(64)
    x = fwd_pass4(x, wt(W, 1, h) * one, wt(W, 2, 2 * h) * one)       # A': stages 1, 2 (uniform)
    x = relayout(x, "A", "B")
    x = fwd_pass4(x, np.array([wt(W, 3, 4 * h + (l >> 4)) for l in L64]),
                  np.array([wt(W, 4, 8 * h + 2 * (l >> 4)) for l in L64]))
    x = relayout(x, "B", "C")
    x = fwd_pass4(x, np.array([wt(W, 5, 16 * h + (l >> 2)) for l in L64]),
                  np.array([wt(W, 6, 32 * h + 2 * (l >> 2)) for l in L64]))
    x = relayout(x, "C", "D")
    x = fwd_pass4(x, np.array([wt(W, 7, 64 * h + l) for l in L64]),
                  np.array([wt(W, 8, 128 * h + 2 * l) for l in L64]))
    return x


def dit_pass4(x, a, b):
    """radix-2 DIT stages at register distance 1 (twiddle a) then 2 (b for (0,2), -i b for (1,3))"""
    x = x.copy()

    def bf(r0, r1, tw):
        t = tw * x[:, r1]
        x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t
    bf(0, 1, a)
    bf(2, 3, a)
    bf(0, 2, b)
    bf(1, 3, -1j * b)
    return x


def e(j, m):
    return np.exp(-2j * np.pi * np.asarray(j, dtype=np.float64) / m)


SIG = e(L64, 2048)                                                 # zeta^-L


def inv_half(Y):
    """Y [64][4] layout D': DIT stages 0..7 inside the half, the lane factor zeta^-L folded into
    pass A' (its u inputs, and its first twiddle); returns layout A' [64][4] (m = L + 64 r')."""
    one = np.ones(64)
    x = dit_pass4(Y, one, one)                                      # D': stages 0, 1 (trivial)
    x = relayout(x, "D", "C")
    x = dit_pass4(x, e(L64 & 3, 8), e(L64 & 3, 16))                 # C': stages 2, 3
    x = relayout(x, "C", "B")
    x = dit_pass4(x, e(L64 & 15, 32), e(L64 & 15, 64))              # B': stages 4, 5
    x = relayout(x, "B", "A")
    x[:, 0::2] = x[:, 0::2] * SIG[:, None]
    return dit_pass4(x, e(L64, 128) * SIG, e(L64, 256))             # A': stages 6, 7


def inv_final(h0, h1):
    """stage 8 over both halves (layout A, n = L + 64 r: pairs (r, r + 4)) and the register
    factors of the post-twist; returns the 1024 real coefficients (re: n, im: n + 512)"""
    x = np.concatenate([h0, h1], axis=1)
    c, c2 = e(L64, 512), e(L64 + 64, 512)
    for r, W in ((0, c), (1, c2), (2, -1j * c), (3, -1j * c2)):
        t = W * x[:, r + 4]
        x[:, r], x[:, r + 4] = x[:, r] + t, x[:, r] - t
    x = x * np.exp(-2j * np.pi * np.arange(8) / 32)[None, :]
    flat = np.empty(512, dtype=complex)
    flat[E.IDX_A] = x
    return np.concatenate([flat.real, flat.imag])


def key_slot_index(h):
    """for each (L, r') of half h in layout D': the v6 key layout's (r6, L6) = (n & 7, n >> 3)"""
    n = 256 * h + IDX["D"]
    return n & 7, n >> 3


def main():
    W, _ = E.twiddles_v6()
    T = E.tables()
    rng = np.random.default_rng(12)
    worst = 0.0
    for t in range(5):
        d = rng.integers(-512, 512, (4, 1024))
        bk = rng.integers(-2**31, 2**31, (4, 1024))
        if t == 4:
            d[:] = 511
        # the key as v6 stores it: layout C [L6][r6] = slot 8 L6 + r6, scaled by 1/512
        keyC = [E.fwd(bk[p].astype(float), T) / 512 for p in range(4)]
        halves = []
        for h in (0, 1):
            r6, l6 = key_slot_index(h)
            acc = np.zeros((64, 4), dtype=complex)
            for p in range(4):
                zA = (d[p, :512] + 1j * d[p, 512:]).astype(complex)[E.IDX_A]
                D = fwd_half(zA, h, W)
                # v6's spectrum, slot for slot
                ref = np.empty(512, dtype=complex)
                ref[E.IDX_C] = E.fwd(d[p].astype(float), T)
                assert np.allclose(D, ref[256 * h + IDX["D"]], atol=1e-6), (t, h, p)
                acc += D * keyC[p][l6, r6]
            halves.append(inv_half(acc))
        c = inv_final(*halves)
        want = sum(E.negacyclic(d[p], bk[p]) for p in range(4))
        assert all(int(g) == int(w) for g, w in zip(np.rint(c).astype(np.int64), want)), t
        worst = max(worst, float(np.max(np.abs(c - np.rint(c)))))
    print(f"emu_v12: half transforms equal v6's spectrum slot for slot; external product exact; "
          f"worst |c - rint(c)| = {worst:.4f}")


if __name__ == "__main__":
    main()
