"""emu_v9.py — numpy emulation of the v9 blind-rotation step (4 waves per ciphertext), layout by
layout, before any HIP: wave q = (w, d) runs v6's forward transform of digit polynomial d of
accumulator polynomial w; wave q = (c, h) then MACs the 4 spectra over half h of the slots of
output c (layout P: slot s = 256 h + 4 L + t) and runs the DIT stages 0..7 of that half in four
radix-4 register passes (layouts P, Q, R, S), the two waves of an output exchange their halves
for stage 8 (each computes the whole output), post-twist zeta^-n, rint.  Checks the result equals
v6's inverse (emu_v6.inv_dit) and the exact negacyclic product, and prints the twiddle tables'
index maps the kernel uses.

    python scripts/emu_v9.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import emu_v6 as E  # noqa: E402

Lv = np.arange(64)


def W(k, j):
    """DIT stage k twiddle for position j < 2^k: e^{-i pi j / 2^k}"""
    return np.exp(-1j * np.pi * np.asarray(j) / (1 << k))


# local slot s' in [0, 256) held by (lane L, register t) in each layout
def lay_P(L, t): return 4 * L + t                          # regs = bits 0, 1
def lay_Q(L, t): return (L & 3) + 4 * t + 16 * (L >> 2)    # regs = bits 2, 3
def lay_R(L, t): return (L & 15) + 16 * t + 64 * (L >> 4)  # regs = bits 4, 5
def lay_S(L, t): return L + 64 * t                         # regs = bits 6, 7


def idx(lay):
    return np.array([[lay(L, t) for t in range(4)] for L in range(64)])


IP, IQ, IR, IS = idx(lay_P), idx(lay_Q), idx(lay_R), idx(lay_S)


def relay(x, src, dst):
    flat = np.empty(256, dtype=complex)
    flat[src] = x
    return flat[dst]


def radix4(x, k, idx_map):
    """DIT stages k (register distance 1) and k + 1 (distance 2) on a [64][4] array whose
    register bits are local-slot bits k, k + 1; twiddles from each element's low slot bits"""
    x = x.copy()
    s = idx_map                                    # [64][4] local slots
    def bf(r0, r1, kk):
        j = s[:, r0] & ((1 << kk) - 1)            # position within the 2^kk block
        t = W(kk, j) * x[:, r1]
        x[:, r0], x[:, r1] = x[:, r0] + t, x[:, r0] - t
    bf(0, 1, k); bf(2, 3, k)
    bf(0, 2, k + 1); bf(1, 3, k + 1)
    return x


def half_inverse(Sp):
    """Sp [64][4] in layout P -> U [64][4] in layout S (local natural order n' = L + 64 t)"""
    x = radix4(Sp, 0, IP)
    x = radix4(relay(x, IP, IQ), 2, IQ)
    x = radix4(relay(x, IQ, IR), 4, IR)
    x = radix4(relay(x, IR, IS), 6, IS)
    return x


def step_v9(Zc):
    """Zc: the summed spectrum of output c, [64][8] in layout C (slot 8L + r) -> 1024 reals"""
    flat = np.empty(512, dtype=complex)
    flat[E.IDX_C] = Zc
    U = []
    for h in range(2):
        Sp = flat[256 * h + IP]
        U.append(half_inverse(Sp))
    n1 = IS                                        # n' = L + 64 t
    V1 = W(8, n1) * U[1]                           # wave h = 1 sends W_8 U1
    X = np.concatenate([U[0] + V1, U[0] - V1], axis=1)   # [64][8]: n = L + 64 r
    n = Lv[:, None] + 64 * np.arange(8)[None, :]
    X = X * np.exp(-1j * np.pi * n / 1024)        # post-twist zeta^-n
    out = np.empty(512, dtype=complex)
    out[n] = X
    return np.concatenate([out.real, out.imag])


def main():
    T = E.tables()
    rng = np.random.default_rng(11)
    worst = 0.0
    for trial in range(6):
        d = rng.integers(-512, 512, (4, 1024))
        bk = rng.integers(-2**31, 2**31, (4, 1024))
        Z = sum(E.fwd(d[p].astype(float), T) * (E.fwd(bk[p].astype(float), T) / 512) for p in range(4))
        c9 = step_v9(Z)
        c6 = E.inv_dit(Z)
        assert np.max(np.abs(c9 - c6)) < 0.2, np.max(np.abs(c9 - c6))   # fp64 rounding noise at |c| ~ 2^48
        want = sum(E.negacyclic(d[p], bk[p]) for p in range(4))
        got = np.rint(c9).astype(np.int64)
        assert all(int(g) == int(w) for g, w in zip(got, want)), trial
        worst = max(worst, float(np.max(np.abs(c9 - np.rint(c9)))))
    print(f"emu_v9: 4-wave split (MAC by halves, radix-4 half inverses, stage-8 exchange) exact; "
          f"worst |c - rint(c)| = {worst:.4f}")
    # twiddle index maps per layout (for the kernel's tables)
    print("Q: stage 2 j = L&3; stage 3 j = (L&3) + 4 (t&1)")
    print("R: stage 4 j = L&15; stage 5 j = (L&15) + 16 (t&1)")
    print("S: stage 6 j = L; stage 7 j = L + 64 (t&1); stage 8 j = L + 64 t")


if __name__ == "__main__":
    main()
