"""Python emulator of the v4 blind-rotation step's index math: forward CT NTT as v2 (negated
twiddles, add3 form), pointwise MAC with REDC (lazy), inverse as a bit-reversed-input DIT
Cooley-Tukey transform in layouts C -> B -> A with a post-twist psi^-n, then the lazy CRT.
Checks one external product against the exact negacyclic product.  Dev tool, not the product."""
import random
N = 1024
Q = [134215681, 134203393]
M32 = 0xFFFFFFFF


def brv(x, b=10):
    return int('{:0{w}b}'.format(x, w=b)[::-1], 2)


def root(q):
    for g in range(2, 1000):
        c = pow(g, (q - 1) // 2048, q)
        if pow(c, 1024, q) == q - 1:
            return c


PSI = [root(q) for q in Q]
IPSI = [pow(p, q - 2, q) for p, q in zip(PSI, Q)]


def sh(w, q):
    return (w << 32) // q


def bf_ct(x, y, w, q, bound):
    """negated-twiddle form: nt = qh q + lo(y wn); x' = u - nt; y' = u + nt + 2q"""
    wn = (-w) & M32
    wp = sh(w, q)
    assert y < 2**32 and x < 2**32
    qh = (y * wp) >> 32
    nt = (qh * q + ((y * wn) & M32)) & M32
    t = (-nt) & M32
    assert t < 2 * q, (t, q)
    x2 = (x - nt) & M32
    y2 = (x + nt + 2 * q) & M32
    assert x2 == x + t and y2 == x - t + 2 * q       # no wrap
    assert x2 % q == (x + w * y) % q and y2 % q == (x - w * y) % q
    return x2, y2


def jA(L, r): return L + 64 * r
def jB(L, r): return (L & 3) | (r << 2) | ((L >> 2) << 6)
def jC(L, r): return 16 * L + r


def relayout(x, src, dst):
    vals = {}
    for L in range(64):
        for r in range(16):
            vals[src(L, r)] = x[L][r]
    return [[vals[dst(L, r)] for r in range(16)] for L in range(64)]


def fwd_ntt(a, s):
    """natural -> bit-reversed, Longa-Naehrig (index space; v2 kernel equivalent)"""
    q = Q[s]
    P = [pow(PSI[s], brv(k), q) for k in range(N)]
    x = list(a)
    t = N
    m = 1
    while m < N:
        t //= 2
        for i in range(m):
            w = P[m + i]
            for j in range(2 * i * t, 2 * i * t + t):
                x[j], x[j + t] = bf_ct(x[j], x[j + t], w, q, None)
        m *= 2
    return x


def tw_inv(s, stage, p):
    q = Q[s]
    return pow(IPSI[s], p << (10 - stage), q)


def inv_v4(Y, s):
    """Y in layout C as [L][r] (slot k = 16L + r): DIT stages 0..3 (C), 4..5 (B), 6..9 (A),
    post-twist; returns layout A values (n = L + 64 r), lazy [0, 2q)."""
    q = Q[s]
    x = [row[:] for row in Y]
    for st in range(4):                      # layout C, uniform twiddles, p = r mod 2^st
        d = 1 << st
        for L in range(64):
            for r in range(16):
                if r & d:
                    continue
                p = r & (d - 1)
                assert jC(L, r) % (1 << st) == p
                if st <= 1 and p == 0:       # twiddle 1: no multiply, offset K
                    K = 4 * q if st == 0 else 8 * q
                    u, v = x[L][r], x[L][r + d]
                    assert v <= K
                    x[L][r], x[L][r + d] = u + v, u + K - v
                    assert x[L][r] < 2**32 and x[L][r + d] < 2**32
                    continue
                x[L][r], x[L][r + d] = bf_ct(x[L][r], x[L][r + d], tw_inv(s, st, p), q, None)
    x = relayout(x, jC, jB)
    for st in (4, 5):                        # layout B, k bit st = r bit (st - 2)
        d = 1 << (st - 2)
        for L in range(64):
            for r in range(16):
                if r & d:
                    continue
                g = r & (d - 1)
                p = (L & 3) | (g << 2)
                assert jB(L, r) % (1 << st) == p and jB(L, r + d) == jB(L, r) + (1 << st)
                x[L][r], x[L][r + d] = bf_ct(x[L][r], x[L][r + d], tw_inv(s, st, p), q, None)
    x = relayout(x, jB, jA)
    for st in range(6, 10):                  # layout A, k bit st = r bit (st - 6)
        d = 1 << (st - 6)
        for L in range(64):
            for r in range(16):
                if r & d:
                    continue
                g = r & (d - 1)
                p = L + 64 * g
                assert jA(L, r) % (1 << st) == p and jA(L, r + d) == jA(L, r) + (1 << st)
                x[L][r], x[L][r + d] = bf_ct(x[L][r], x[L][r + d], tw_inv(s, st, p), q, None)
    for L in range(64):                      # post-twist psi^-n, n = L + 64 r (Shoup lazy, positive)
        for r in range(16):
            n = L + 64 * r
            w = pow(IPSI[s], n, q)
            y = x[L][r]
            assert y < 2**32
            qh = (y * sh(w, q)) >> 32
            t = (y * w - qh * q) & M32
            assert t < 2 * q and t % q == y * w % q
            x[L][r] = t
    return x


def crt_lazy(x0, x1):
    q0, q1 = Q
    h = pow(q0, q1 - 2, q1)
    d = (x1 + 3 * q1 - x0) & M32
    assert x1 + 3 * q1 - x0 > 0 and d < 2**32
    qh = (d * sh(h, q1)) >> 32
    t = (d * h - qh * q1) & M32
    assert t < 2 * q1
    t = min(t, (t - q1) & M32)
    tc = t - q1 if t > (q1 - 1) // 2 else t
    return (x0 + q0 * tc) & M32


def main():
    rnd = random.Random(1)
    # 4 digit polys in [-512, 511] and 4 BK rows (Torus32), one output poly c
    D = [[rnd.randrange(-512, 512) for _ in range(N)] for _ in range(4)]
    Bk = [[rnd.randrange(0, 2**32) for _ in range(N)] for _ in range(4)]
    exact = [0] * N
    for p in range(4):
        for i in range(N):
            di = D[p][i]
            if di == 0:
                continue
            for j in range(N):
                k = i + j
                v = di * Bk[p][j]
                if k >= N:
                    exact[k - N] -= v
                else:
                    exact[k] += v
    exact = [e & M32 for e in exact]
    outs = []
    for s in range(2):
        q = Q[s]
        Dh = [fwd_ntt([(d + q) for d in D[p]], s) for p in range(4)]            # lifted digits
        assert max(max(v) for v in Dh) < 22 * q
        ninv = pow(N, q - 2, q)
        R = (1 << 32) % q
        Bh = [[(v * ninv % q) * R % q for v in fwd_ntt([b % q for b in Bk[p]], s)] for p in range(4)]
        qinv_neg = (-pow(q, -1, 1 << 32)) & M32
        Y = []
        for k in range(N):
            xx = sum(Dh[p][k] * Bh[p][k] for p in range(4))
            assert xx < 2**61
            m = (xx * qinv_neg) & M32
            t = (xx + m * q) >> 32
            assert t < 3.75 * q + 1
            Y.append(t)
        YC = [[Y[jC(L, r)] for r in range(16)] for L in range(64)]
        outs.append(inv_v4(YC, s))
    got = [0] * N
    for L in range(64):
        for r in range(16):
            got[L + 64 * r] = crt_lazy(outs[0][L][r], outs[1][L][r])
    bad = sum(1 for a, b in zip(got, exact) if a != b)
    print("mismatches:", bad)
    assert bad == 0


if __name__ == "__main__":
    main()
