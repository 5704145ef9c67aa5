"""Stage-by-stage check of one v2 CMux step on the GPU (scripts/libv2dbg.so) against the
emulator (scripts/emu_v2.py) and the oracle.  Dev tool."""
import ctypes, os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE); sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import emu_v2 as E
import oracle_ctypes as O
lib = ctypes.CDLL(os.path.join(HERE, "libv2dbg.so"))
N = 1024
rng = np.random.default_rng(5)
acc = rng.integers(-2**31, 2**31, (2, N), dtype=np.int64).astype(np.int32)
bk0 = rng.integers(-2**31, 2**31, (4, 2, N), dtype=np.int64).astype(np.int32)
a = 77
accio = acc.copy()
dump_all = np.zeros(2 * 16 * N + 2 * N, np.uint32)
dump = dump_all[:2 * 16 * N].reshape(2, 16, N)
P = lambda x: x.ctypes.data_as(ctypes.c_void_p)
lib.run_staged(P(accio), a, P(bk0), P(dump_all))
M32 = 0xFFFFFFFF
accu = acc.astype(np.int64) & M32
for s in range(2):
    q = E.Q[s]
    dig = []
    for c in range(2):
        d0 = []; d1 = []
        for j in range(N):
            si = (j - a) & 2047; v = int(accu[c][si & 1023]); rot = (-v) & M32 if si & 1024 else v
            t = (rot - int(accu[c][j]) + 2149580800) & M32
            d0.append((((t >> 22) & 1023) - 512) % q); d1.append((((t >> 12) & 1023) - 512) % q)
        dig += [d0, d1]
    print(f"prime {s} digits  ok:", [list(dump[s][p]) == dig[p] for p in range(4)])
    f = [E.ref_fwd(dig[p], s) for p in range(4)]
    print(f"prime {s} forward ok:", [list(dump[s][4 + p]) == f[p] for p in range(4)],
          [int(np.sum(np.array(dump[s][4 + p], np.int64) != np.array(f[p]))) for p in range(4)])
    scale = pow(N, q - 2, q) * ((1 << 32) % q) % q
    bkn = {(p, c): [v * scale % q for v in E.ref_fwd([int(x) for x in bk0[p, c]], s)] for p in range(4) for c in range(2)}
    rinv = pow((1 << 32) % q, q - 2, q)
    mac = [[sum(f[p][j] * bkn[(p, c)][j] for p in range(4)) * rinv % q for j in range(N)] for c in range(2)]
    print(f"prime {s} MAC ok:", [list(dump[s][8 + c]) == mac[c] for c in range(2)],
          [int(np.sum(np.array(dump[s][8 + c], np.int64) != np.array(mac[c]))) for c in range(2)])
fullbk = np.zeros((500, 4, 2, N), np.int32); fullbk[0] = bk0
ok = O.OracleKey(fullbk, None, use_ntt=False)
want = ok.mux_rotate(acc, 0, a)
print("final (debug kernel) ok:", np.array_equal(accio, want), int(np.sum(accio != want)))
staged = dump_all[2 * 16 * N:].view(np.int32).reshape(2, N)
print("final (staged kernel) ok:", np.array_equal(staged, want), int(np.sum(staged != want)))
print("crt_h", dump[0][14][0], dump[0][14][1], "reduced<q:", [(dump[s][12 + c] < E.Q[s]).all() for s in range(2) for c in range(2)])
q0, q1 = E.Q
x0 = dump[0][12].astype(np.int64); x1 = dump[1][12].astype(np.int64)
exp = np.array([E.crt(int(a_), int(b_)) for a_, b_ in zip(x0, x1)], np.int64)
print("host crt of device residues == want-acc:", np.array_equal((exp + (acc[0].astype(np.int64) & 0xFFFFFFFF)) & 0xFFFFFFFF, want[0].astype(np.int64) & 0xFFFFFFFF))
def ref_inv(a, s):
    q = E.Q[s]; a = list(a); t = 1; m = N
    IP = E.tabs[s]['ipsi']
    while m > 1:
        h = m // 2; j1 = 0
        for i in range(h):
            S = IP[h + i]
            for j in range(j1, j1 + t):
                U = a[j]; V = a[j + t]; a[j] = (U + V) % q; a[j + t] = (U - V) * S % q
            j1 += 2 * t
        t *= 2; m //= 2
    return a
for s in range(2):
    q = E.Q[s]
    dig = []
    for c in range(2):
        d0 = []; d1 = []
        for j in range(N):
            si = (j - a) & 2047; v = int(accu[c][si & 1023]); rot = (-v) & M32 if si & 1024 else v
            t = (rot - int(accu[c][j]) + 2149580800) & M32
            d0.append((((t >> 22) & 1023) - 512) % q); d1.append((((t >> 12) & 1023) - 512) % q)
        dig += [d0, d1]
    f = [E.ref_fwd(dig[p], s) for p in range(4)]
    scale = pow(N, q - 2, q) * ((1 << 32) % q) % q
    bkn = {(p, c): [v * scale % q for v in E.ref_fwd([int(x) for x in bk0[p, c]], s)] for p in range(4) for c in range(2)}
    rinv = pow((1 << 32) % q, q - 2, q)
    mac = [[sum(f[p][j] * bkn[(p, c)][j] for p in range(4)) * rinv % q for j in range(N)] for c in range(2)]
    inv = [ref_inv(mac[c], s) for c in range(2)]
    print(f"prime {s} inverse ok:", [list(dump[s][10 + c]) == inv[c] for c in range(2)],
          [int(np.sum(np.array(dump[s][10 + c], np.int64) != np.array(inv[c]))) for c in range(2)])
    # emulator inverse on the device MAC output, layout C -> A
    x = [[[int(dump[s][8 + c][16 * L + r]) for r in range(16)] for L in range(64)] for c in range(2)]
    y = E.ntt_inv(x, s)
    emu = [[None] * N for _ in range(2)]
    for c in range(2):
        for L in range(64):
            for r in range(16): emu[c][L + 64 * r] = y[c][L][r] % q
    print(f"prime {s} emulator-inverse == ref:", [emu[c] == inv[c] for c in range(2)])
