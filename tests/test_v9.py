"""The 4-wave blind rotation (csrc/blind_rotate_v9.hip), forced onto every launch
with TFHE_AMD_V9=2 in a subprocess (the policy is read once per process), against the exact CPU
oracle, Torus32 for Torus32: raw CMux steps at the rotation edges and every register shift,
gate batches across the sizes its launch policy covers (1 ... 2 CUs) incl. the launch's ragged
ends, MUX halves, woKS with zero rotations, circuit rows (three-input MAJ / XOR3), and the
guard's forced fallback.  CPU: the emulation of its data flow (scripts/emu_v9.py)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_v9_data_flow_emulation():
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "emu_v9.py")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "exact" in r.stdout


CODE = r"""
import sys, numpy as np, torch
sys.path[:0] = [%r, %r]
import tfhe_amd as T, oracle_ctypes as O
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); o = O.OracleKey(K.bk, K.ksk)
rng = np.random.default_rng(9)
def enc(bits):
    return K.encrypt(np.asarray(bits), rng)
# raw CMux steps (k_blind_rotate_v9_debug through TFHE_AMD_BR=9)
T.select_kernel(9)
B, iters = 4, 32
acc0 = rng.integers(-2**31, 2**31, (B, 2, 1024), dtype=np.int64).astype(np.int32)
bara = rng.integers(0, 2049, (B, iters), dtype=np.int64).astype(np.int32)
bara[0, :10] = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048]
bara[1, :10] = [127, 128, 129, 960, 1087, 1088, 1984, 2000, 31, 32]
q = np.arange(32)
bara[2] = 64 * q + np.mod(7 * q, 64)
bara[3] = 64 * q + 63 - q
d_acc = torch.from_numpy(acc0.copy()).cuda()
c.blind_rotate_dev(d_acc, torch.from_numpy(bara).cuda(), iters); c.sync()
assert "v9" in ",".join(c.last_kernels()), c.last_kernels()
got = d_acc.cpu().numpy()
for b in range(B):
    want = acc0[b].copy()
    for i in range(iters):
        if bara[b, i] != 0:
            want = o.mux_rotate(want, i, int(bara[b, i]))
    assert np.array_equal(got[b], want), ("cmux", b)
T.select_kernel(0)
# gate batches: every output decrypts; sampled outputs (launch ends and random) vs the oracle
for gate, B in (("NAND", 1), ("XOR", 7), ("AND", 64), ("ORYN", 256), ("NAND", 300), ("XNOR", 512)):
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = enc(x), enc(y)
    r_a, r_b = c.gate_host(gate, a_a, a_b, b_a, b_b)
    assert any("v9" in k for k in c.last_kernels()), c.last_kernels()
    idx = np.unique(np.concatenate([[0, B - 1, B // 2], rng.choice(B, min(B, 12), replace=False)]))
    w_a, w_b = o.gate_batch(gate, a_a[idx], a_b[idx], b_a[idx], b_b[idx])
    assert np.array_equal(r_a[idx], w_a) and np.array_equal(r_b[idx], w_b), (gate, B)
    f = {"NAND": lambda u, v: 1 - (u & v), "XOR": lambda u, v: u ^ v, "AND": lambda u, v: u & v,
         "ORYN": lambda u, v: u | (1 - v), "XNOR": lambda u, v: 1 - (u ^ v)}[gate]
    assert np.array_equal(K.decrypt(r_a, r_b), f(x, y)), (gate, B)
# MUX (two blind rotations per gate in one launch)
B = 40
s, u, v = (rng.integers(0, 2, B) for _ in range(3))
(sa, sb), (ua, ub), (va, vb) = enc(s), enc(u), enc(v)
m_a, m_b = c.gate_host("MUX", sa, sb, ua, ub, va, vb)
w_a, w_b = o.gate_batch("MUX", sa, sb, ua, ub, va, vb)
assert np.array_equal(m_a, w_a) and np.array_equal(m_b, w_b), "mux"
# woKS with zero rotations (a = 0 steps skipped by the whole workgroup)
x_a = rng.integers(-2**31, 2**31, (6, 500), dtype=np.int64).astype(np.int32)
x_a[0] = 0
x_a[1, ::2] = 0
x_b = rng.integers(-2**31, 2**31, 6, dtype=np.int64).astype(np.int32)
g_a, g_b = c.woks_host(1 << 29, x_a, x_b)
for k in range(6):
    e_a, e_b = o.bootstrap_woks(1 << 29, x_a[k], x_b[k])
    assert np.array_equal(g_a[k], e_a) and g_b[k] == e_b, ("woks", k)
# circuit rows: a full adder level (XOR3 + MAJ rows), 8-bit ripple add, decrypted
C = T.Circuit()
a8, b8 = C.inputs(8), C.inputs(8)
s8, co = C.add(a8, b8)
Bc = 33
xa_, ya_ = rng.integers(0, 256, Bc), rng.integers(0, 256, Bc)
inp = {**dict(zip(a8, T.bits_of(xa_, 8))), **dict(zip(b8, T.bits_of(ya_, 8)))}
got = C.run(c, Bc, inp, s8 + [co], K, rng)
assert any("v9_rows" in k for k in c.last_kernels()), c.last_kernels()
assert np.array_equal(T.int_of([got[w] for w in s8 + [co]]), xa_ + ya_), "circuit"
# the guard's fallback forced (threshold 0): every v9 output recomputed exactly, outputs unchanged
T.set_guard_threshold(0.0)
B = 20
x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
(a_a, a_b), (b_a, b_b) = enc(x), enc(y)
c.guard_stats(reset=True)
r_a, r_b = c.gate_host("NAND", a_a, a_b, b_a, b_b)
d, rec = c.guard_stats()
w_a, w_b = o.gate_batch("NAND", a_a, a_b, b_a, b_b)
assert rec == B and np.array_equal(r_a, w_a) and np.array_equal(r_b, w_b), ("guard", rec)
T.set_guard_threshold(0.125)
c.guard_stats(reset=True)
r_a, r_b = c.gate_host("NAND", a_a, a_b, b_a, b_b)
d, rec = c.guard_stats()
assert rec == 0 and d < 0.125 and np.array_equal(r_a, w_a), ("guard default", d, rec)
print("v9 ok, largest distance", d)
""" % (os.path.join(REPO, "cpu-gpu-tfhe_amd"), os.path.join(REPO, "tests"))


@pytest.mark.gpu
def test_v9_bit_exact_subprocess():
    env = dict(os.environ, TFHE_AMD_V9="2")
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "v9 ok" in r.stdout
