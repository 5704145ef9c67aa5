"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, Torus32 bit-exact
(SURVEY.md §8(c) P1), plus decryption truth tables (P2)."""
import ctypes
import os

import numpy as np
import pytest

import oracle_ctypes as O
import tfhe_amd as T

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N, n = 1024, 500
TRUTH = {
    "NAND": lambda x, y: 1 - (x & y), "OR": lambda x, y: x | y, "AND": lambda x, y: x & y,
    "XOR": lambda x, y: x ^ y, "XNOR": lambda x, y: 1 - (x ^ y), "NOR": lambda x, y: 1 - (x | y),
    "ANDNY": lambda x, y: (1 - x) & y, "ANDYN": lambda x, y: x & (1 - y),
    "ORNY": lambda x, y: (1 - x) | y, "ORYN": lambda x, y: x | (1 - y),
}


def _torch():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def test_blind_rotate_steps_match_oracle(ctx, okey, rng):
    """A few CMux steps (rotation + decomposition + exact NTT product + CRT) on explicit
    accumulators, including the rotation edge cases 0 (skip), 1, N-1, N, N+1, 2N-1, 2N."""
    torch = _torch()
    B, iters = 6, 8
    acc0 = rng.integers(-2**31, 2**31, (B, 2, N), dtype=np.int64).astype(np.int32)
    bara = rng.integers(0, 2049, (B, iters), dtype=np.int64).astype(np.int32)
    bara[0] = [0, 1, 1023, 1024, 1025, 2047, 2048, 5]
    bara[1] = 2048
    bara[2, :4] = 0
    d_acc = torch.from_numpy(acc0.copy()).cuda()
    d_bara = torch.from_numpy(bara).cuda()
    ctx.blind_rotate_dev(d_acc, d_bara, iters)
    ctx.sync()
    got = d_acc.cpu().numpy()
    for b in range(B):
        want = acc0[b].copy()
        for i in range(iters):
            if bara[b, i] != 0:
                want = okey.mux_rotate(want, i, int(bara[b, i]))
        assert np.array_equal(got[b], want), f"ciphertext {b}"


@pytest.mark.parametrize("gate", list(TRUTH))
def test_gate_batch_bit_exact(ctx, okey, keyset, rng, gate):
    B = 16
    x = rng.integers(0, 2, B)
    y = rng.integers(0, 2, B)
    a_a, a_b = keyset.encrypt(x, rng)
    b_a, b_b = keyset.encrypt(y, rng)
    r_a, r_b = ctx.gate_host(gate, a_a, a_b, b_a, b_b)
    o_a, o_b = okey.gate_batch(gate, a_a, a_b, b_a, b_b)
    assert np.array_equal(r_a, o_a) and np.array_equal(r_b, o_b)
    assert np.array_equal(keyset.decrypt(r_a, r_b), TRUTH[gate](x, y))


def test_mux_bit_exact(ctx, okey, keyset, rng):
    B = 16
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    r_a, r_b = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
    o_a, o_b = okey.gate_batch("MUX", sa, sb, xa, xb, ya, yb)
    assert np.array_equal(r_a, o_a) and np.array_equal(r_b, o_b)
    assert np.array_equal(keyset.decrypt(r_a, r_b), np.where(s == 1, x, y))


def test_woks_and_keyswitch_bit_exact(ctx, okey, keyset, rng):
    B = 8
    x_a = rng.integers(-2**31, 2**31, (B, n), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    x_b[0] = np.int32(-2**20 + 5)      # modSwitch wrap edge: barb = 0
    x_a[1, :50] = np.int32(-(2**20))   # bara = 0 through the wrap on a run of keys
    x_a[2, :50] = 0                    # bara = 0 (skipped CMux)
    u_a, u_b = ctx.woks_host(T.MU, x_a, x_b)
    o_a, o_b = okey.woks_batch(T.MU, x_a, x_b)
    assert np.array_equal(u_a, o_a) and np.array_equal(u_b, o_b)
    k_a, k_b = ctx.keyswitch_host(u_a, u_b)
    ko_a, ko_b = okey.keyswitch_batch(o_a, o_b)
    assert np.array_equal(k_a, ko_a) and np.array_equal(k_b, ko_b)
    r_a, r_b = ctx.bootstrap_host(T.MU, x_a, x_b)
    assert np.array_equal(r_a, ko_a) and np.array_equal(r_b, ko_b)


def test_keyswitch_random_inputs(ctx, okey, rng):
    B = 5
    u_a = rng.integers(-2**31, 2**31, (B, N), dtype=np.int64).astype(np.int32)
    u_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    u_a[0] = 0                          # every digit of aibar = 2^15 is 0 except none
    k_a, k_b = ctx.keyswitch_host(u_a, u_b)
    o_a, o_b = okey.keyswitch_batch(u_a, u_b)
    assert np.array_equal(k_a, o_a) and np.array_equal(k_b, o_b)


def test_kernel_generations_agree(ctx, keyset, rng):
    """Both blind-rotation generations the library carries (v4 exact NTT and v6 fp64 FFT, whose
    rounded products equal the exact ones) give identical Torus32 results on the same gates and
    on explicit CMux steps."""
    torch = _torch()
    B, iters = 8, 6
    x = rng.integers(0, 2, B)
    y = rng.integers(0, 2, B)
    a_a, a_b = keyset.encrypt(x, rng)
    b_a, b_b = keyset.encrypt(y, rng)
    acc0 = rng.integers(-2**31, 2**31, (B, 2, N), dtype=np.int64).astype(np.int32)
    bara = rng.integers(0, 2048, (B, iters), dtype=np.int64).astype(np.int32)
    default = T.version()
    gens = T.available_kernels()
    assert 4 in gens and 6 in gens, gens
    outs = {}
    try:
        for v in gens:
            T.select_kernel(v)
            d_acc = torch.from_numpy(acc0.copy()).cuda()
            ctx.blind_rotate_dev(d_acc, torch.from_numpy(bara).cuda(), iters)
            ctx.sync()
            outs[v] = (ctx.gate_host("XOR", a_a, a_b, b_a, b_b), d_acc.cpu().numpy())
    finally:
        tag = default.split("br-v")[1].split(" ")[0]
        T.select_kernel(int(tag) if tag.isdigit() else 0)
    for v in gens:
        (ra, rb), acc = outs[v]
        (ra4, rb4), acc4 = outs[4]
        assert np.array_equal(ra, ra4) and np.array_equal(rb, rb4), v
        assert np.array_equal(acc, acc4), v
    assert np.array_equal(keyset.decrypt(*outs[4][0]), x ^ y)


def test_chunk_boundaries_bit_exact(ctx, okey, keyset, rng):
    """Launches larger than one round of workgroups (4 per CU: 1024 ciphertexts on 256 CUs) are
    split into one-round launches; the ciphertexts on both sides of every split, and of the MUX
    halves (2B rotations in one launch), match the oracle bit for bit."""
    B = 1100
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    r_a, r_b = ctx.gate_host("NAND", a_a, a_b, b_a, b_b)
    assert np.array_equal(keyset.decrypt(r_a, r_b), 1 - (x & y))
    idx = np.array([0, 1, 1022, 1023, 1024, 1025, 1099])
    o_a, o_b = okey.gate_batch("NAND", a_a[idx], a_b[idx], b_a[idx], b_b[idx])
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)
    B = 600                                   # MUX: 1200 rotations, split at 1024 (inside half 1)
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    r_a, r_b = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
    assert np.array_equal(keyset.decrypt(r_a, r_b), np.where(s == 1, x, y))
    idx = np.array([0, 423, 424, 425, 599])   # half-1 rotation 424 is ciphertext 1024
    o_a, o_b = okey.gate_batch("MUX", sa[idx], sb[idx], xa[idx], xb[idx], ya[idx], yb[idx])
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)


def test_paired_workgroups_bit_exact(ctx, okey, keyset, rng):
    """Launches of CUs < n <= 2 CUs ciphertexts (256 CUs) run two ciphertexts per workgroup
    (k_blind_rotate_v6p, whose waves meet per ciphertext through LDS step counters): an odd count
    (a padding ciphertext that writes nothing), MUX halves meeting inside one workgroup, and
    a_i = 0 steps, which the paired kernel runs as identity CMuxes instead of skipping — every
    output against the oracle."""
    B = 301
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    r_a, r_b = ctx.gate_host("AND", a_a, a_b, b_a, b_b)
    kern = ctx.last_kernels()
    o_a, o_b = okey.gate_batch("AND", a_a, a_b, b_a, b_b)
    assert np.array_equal(r_a, o_a) and np.array_equal(r_b, o_b)   # parity first, then which kernel
    assert any("v6p(paired+reg-rotation+pair-sync)" in k for k in kern), kern
    B = 199                                   # MUX: 398 rotations; rotations 198 | 199 share a workgroup
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    r_a, r_b = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
    o_a, o_b = okey.gate_batch("MUX", sa, sb, xa, xb, ya, yb)
    assert np.array_equal(r_a, o_a) and np.array_equal(r_b, o_b)
    B = 300
    x_a = rng.integers(-2**31, 2**31, (B, n), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    x_a[::3, :40] = 0                         # runs of bara = 0 in every third ciphertext
    x_a[1::7, 100:140] = np.int32(-(2**20))   # bara = 0 through the wrap
    u_a, u_b = ctx.woks_host(T.MU, x_a, x_b)
    o_a, o_b = okey.woks_batch(T.MU, x_a, x_b)
    assert np.array_equal(u_a, o_a) and np.array_equal(u_b, o_b)


def test_device_api_rejects_bad_tensors(ctx):
    """Shapes, dtypes, missing MUX inputs and tensors on another GPU are refused on the host,
    before any launch."""
    torch = _torch()
    B = 4
    a = torch.zeros((B, n), dtype=torch.int32, device="cuda")
    b = torch.zeros(B, dtype=torch.int32, device="cuda")
    short = torch.zeros((B - 1, n), dtype=torch.int32, device="cuda")
    with pytest.raises(T.TfheAmdError):
        ctx.gate_dev("NAND", short, b, a, b, a, b)
    with pytest.raises(T.TfheAmdError):
        ctx.gate_dev("NAND", a, b, a.to(torch.int64), b, a, b)
    with pytest.raises(T.TfheAmdError):
        ctx.gate_dev("MUX", a, b, a, b, a, b)
    with pytest.raises(T.TfheAmdError):
        ctx.blind_rotate_dev(torch.zeros((B, 2, N), dtype=torch.int32, device="cuda"),
                             torch.zeros((B, 3), dtype=torch.int32, device="cuda"), 4)
    if torch.cuda.device_count() > 1:   # a tensor on another GPU than the context's
        other = torch.zeros((B, n), dtype=torch.int32, device="cuda:1")
        with pytest.raises(T.TfheAmdError):
            ctx.gate_dev("NAND", a, b, other, b, a, b)


def test_empty_batch_is_a_no_op(ctx, keyset, rng):
    torch = _torch()
    e2 = torch.empty((0, n), dtype=torch.int32, device="cuda")
    e1 = torch.empty(0, dtype=torch.int32, device="cuda")
    ctx.gate_dev("NAND", e2, e1, e2, e1, e2, e1)
    ctx.sync()
    x = rng.integers(0, 2, 3)
    a_a, a_b = keyset.encrypt(x, rng)
    r_a, r_b = ctx.gate_host("NOR", a_a, a_b, a_a, a_b)   # the context still works afterwards
    assert np.array_equal(keyset.decrypt(r_a, r_b), 1 - x)


@pytest.mark.parametrize("B", [1, 12, 13, 96, 255, 256, 257, 400, 768, 769, 1025])
def test_keyswitch_paths_bit_exact(ctx, okey, rng, B):
    """Each key-switch path at and around its threshold: small batch <= 12 (per-key-index
    workgroups, atomic partials), above it the int8 MFMA key switch (ks-v5; 256 ciphertexts per
    workgroup: ragged last tile at 13 / 255 / 257 / 400 / 769 / 1025; key-index split 8 up to
    256, 4 up to 512, 2 up to 1024, none above)."""
    u_a = rng.integers(-2**31, 2**31, (B, N), dtype=np.int64).astype(np.int32)
    u_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    k_a, k_b = ctx.keyswitch_host(u_a, u_b)
    o_a, o_b = okey.keyswitch_batch(u_a, u_b)
    assert np.array_equal(k_a, o_a) and np.array_equal(k_b, o_b)


def test_mux_split_keyswitch(ctx, okey, keyset, rng):
    """MUX key-switches u1 + u2 + (0, 1/8): the two-input form through the split path."""
    B = 300
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    r_a, r_b = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
    assert np.array_equal(keyset.decrypt(r_a, r_b), np.where(s == 1, x, y))
    idx = np.array([0, 150, 299])
    o_a, o_b = okey.gate_batch("MUX", sa[idx], sb[idx], xa[idx], xb[idx], ya[idx], yb[idx])
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)


def test_host_batch_slices(ctx, okey, keyset, rng):
    """Host-pointer batches above one round are pipelined in slices of 1024 (one contiguous input
    copy per slice on a copy stream, the result copy behind each key switch); a 3-input MUX batch
    of 2 100 (slices 1024 / 1024 / 52) decrypts right and matches the oracle at every slice seam;
    a one-round batch of 777 (copied in as two halves) in place."""
    B = 2100
    s, x, y = (rng.integers(0, 2, B) for _ in range(3))
    (sa, sb), (xa, xb), (ya, yb) = (keyset.encrypt(v, rng) for v in (s, x, y))
    r_a, r_b = ctx.gate_host("MUX", sa, sb, xa, xb, ya, yb)
    assert np.array_equal(keyset.decrypt(r_a, r_b), np.where(s == 1, x, y))
    idx = np.array([0, 1023, 1024, 2047, 2048, 2099])
    o_a, o_b = okey.gate_batch("MUX", sa[idx], sb[idx], xa[idx], xb[idx], ya[idx], yb[idx])
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)
    # one round, staged and copied in as two row halves (B > 512): the halves' seam and ends, and
    # in place (the result arrays are the first input's)
    B = 777
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (xa, xb), (ya, yb) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    idx = np.array([0, 387, 388, 389, 776])
    o_a, o_b = okey.gate_batch("XOR", xa[idx], xb[idx], ya[idx], yb[idx])
    r_a, r_b = ctx.gate_host("XOR", xa, xb, ya, yb, out=(xa, xb))
    assert np.array_equal(keyset.decrypt(r_a, r_b), x ^ y)
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)


def test_host_trace_subprocess(keyset, rng, tmp_path):
    """TFHE_AMD_HOST_TRACE=1 (read once per process): one stderr line per host-pointer batch call with
    its host-side phases (staged, sliced and pinned paths), and the results are unchanged."""
    import subprocess
    import sys
    x, y = rng.integers(0, 2, 1100), rng.integers(0, 2, 1100)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    np.savez(tmp_path / "in.npz", a_a=a_a, a_b=a_b, b_a=b_a, b_b=b_b, x=x, y=y)
    code = r"""
import sys, numpy as np
sys.path[:0] = [%r]
import tfhe_amd as T
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); z = np.load(%r)
for B in (64, 1100):
    r = c.gate_host("NAND", z["a_a"][:B], z["a_b"][:B], z["b_a"][:B], z["b_b"][:B])
    assert np.array_equal(K.decrypt(*r), 1 - (z["x"][:B] & z["y"][:B]))
pin = [T.host_copy(z[k][:64]) for k in ("a_a", "a_b", "b_a", "b_b")]
r = c.gate_host("NAND", *pin, out=(T.host_empty((64, 500)), T.host_empty(64)))
assert np.array_equal(K.decrypt(*r), 1 - (z["x"][:64] & z["y"][:64]))
print("trace ok")
""" % (os.path.join(REPO, "cpu-gpu-tfhe_amd"), str(tmp_path / "in.npz"))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, TFHE_AMD_HOST_TRACE="1"),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "trace ok" in r.stdout, r.stdout + r.stderr
    lines = [ln for ln in r.stderr.splitlines() if ln.startswith("host_trace ")]
    assert len(lines) >= 3, r.stderr[-2000:]
    assert any("B=64" in ln for ln in lines) and any("B=1100" in ln for ln in lines)
    assert any(ln.startswith("host_trace pinned ") for ln in lines), lines
    for ln in lines:
        f = dict(kv.split("=") for kv in ln.split()[2:])
        assert float(f["total"]) > 0.0 and all(float(v) >= 0.0 for v in f.values()), ln


@pytest.mark.parametrize("gate,B", [("NAND", 64), ("NAND", 1024), ("MUX", 2100), ("AND", 777)])
def test_pinned_host_batch_equals_device_path(ctx, okey, keyset, rng, gate, B):
    """Caller-owned pinned arrays (tfhe_amd_host_alloc via T.host_copy / host_empty): the host call
    DMAs straight from and into them (no staging).  Every output word equals the device path's on the
    same inputs and the staged host path's; the slice seams match the oracle; then in place (results
    into the first input's pinned arrays); and a call with one array not pinned takes the staged path
    with the same results."""
    torch = _torch()
    nin = 3 if gate == "MUX" else 2
    bits = [rng.integers(0, 2, B) for _ in range(nin)]
    host = [v for b in bits for v in keyset.encrypt(b, rng)]
    pin = [T.host_copy(v) for v in host]
    assert all(T.is_pinned(p) for p in pin) and not T.is_pinned(host[0])
    out = (T.host_empty((B, n)), T.host_empty(B))
    r_a, r_b = ctx.gate_host(gate, *pin, out=out)
    dev = [torch.from_numpy(v).cuda() for v in host]
    d_a = torch.empty((B, n), dtype=torch.int32, device="cuda")
    d_b = torch.empty(B, dtype=torch.int32, device="cuda")
    ctx.reserve(B)
    ctx.gate_dev(gate, d_a, d_b, *dev)
    ctx.sync()
    w_a, w_b = d_a.cpu().numpy(), d_b.cpu().numpy()
    assert np.array_equal(r_a, w_a) and np.array_equal(r_b, w_b)
    s_a, s_b = ctx.gate_host(gate, *host)                   # staged (pageable arrays)
    assert np.array_equal(s_a, w_a) and np.array_equal(s_b, w_b)
    idx = np.unique(np.array([0, B // 2, B - 1] + [i for i in (1023, 1024, 2047, 2048) if i < B]))
    o_a, o_b = okey.gate_batch(gate, *[h[idx] for h in host])
    assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b)
    # in place: the results overwrite the first input's pinned arrays
    r2 = ctx.gate_host(gate, *pin, out=(pin[0], pin[1]))
    assert r2[0] is pin[0] and np.array_equal(pin[0], w_a) and np.array_equal(pin[1], w_b)
    # one input pageable: the staged path, same words
    mixed = [T.host_copy(v) for v in host]
    mixed[2] = host[2].copy()
    m_a, m_b = ctx.gate_host(gate, *mixed, out=(T.host_empty((B, n)), T.host_empty(B)))
    assert np.array_equal(m_a, w_a) and np.array_equal(m_b, w_b)


def test_large_ragged_batch(ctx, okey, keyset, rng):
    """A batch of 12 289 gates: twelve one-round blind-rotation launches plus a ragged 13th
    of one ciphertext, one key switch over all of them; every output decrypts right and the
    ciphertexts at the launch seams match the oracle bit for bit."""
    torch = _torch()
    B = 12 * 1024 + 1
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
    dev = [torch.from_numpy(v).cuda() for v in host]
    r_a = torch.empty((B, n), dtype=torch.int32, device="cuda")
    r_b = torch.empty(B, dtype=torch.int32, device="cuda")
    ctx.reserve(B)
    ctx.gate_dev("XNOR", r_a, r_b, *dev)
    ctx.sync()
    ra, rb = r_a.cpu().numpy(), r_b.cpu().numpy()
    assert np.array_equal(keyset.decrypt(ra, rb), 1 - (x ^ y))
    a_a, a_b, b_a, b_b = host
    idx = np.array([0, 1023, 1024, 6143, 6144, 12287, 12288])
    o_a, o_b = okey.gate_batch("XNOR", a_a[idx], a_b[idx], b_a[idx], b_b[idx])
    assert np.array_equal(ra[idx], o_a) and np.array_equal(rb[idx], o_b)


def test_scratch_reuse_across_streams(ctx, okey, keyset, rng):
    """Two device-API batches on one context from two streams, enqueued back to back with no
    host sync: the engine orders the reuse of its scratch (extracted samples) between the
    streams, so both come out right (truth tables, a sample bit-exact against the oracle)."""
    torch = _torch()
    B = 768
    ctx.reserve(B)
    jobs = []
    for gate in ("NAND", "XOR"):
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        host = keyset.encrypt(x, rng) + keyset.encrypt(y, rng)
        dev = [torch.from_numpy(v).cuda() for v in host]
        out = (torch.empty((B, n), dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda"))
        jobs.append((gate, torch.cuda.Stream(), x, y, host, dev, out))
    torch.cuda.synchronize()
    for gate, st, _, _, _, dev, (r_a, r_b) in jobs:
        ctx.gate_dev(gate, r_a, r_b, *dev, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for gate, _, x, y, (a_a, a_b, b_a, b_b), _, (r_a, r_b) in jobs:
        ra, rb = r_a.cpu().numpy(), r_b.cpu().numpy()
        assert np.array_equal(keyset.decrypt(ra, rb), TRUTH[gate](x, y)), gate
        idx = rng.choice(B, 12, replace=False)
        o_a, o_b = okey.gate_batch(gate, a_a[idx], a_b[idx], b_a[idx], b_b[idx])
        assert np.array_equal(ra[idx], o_a) and np.array_equal(rb[idx], o_b), gate


def test_context_key_memory_and_init(keyset):
    """Product builds hold only the key domains their kernels read: the FFT-domain key (v6),
    the NTT-domain key (v4, the exactness guard's fallback) and the two key-switching layouts
    (the int8 MFMA key switch's signed key bytes, 67 MB, and the small-batch kernel's rows) —
    about 182 MB per cloud key and GPU."""
    import time
    t0 = time.perf_counter()
    c = T.Context(keyset.bk, keyset.ksk, device=0)
    c.sync()
    init_s = time.perf_counter() - t0
    kb = c.key_bytes()
    c.close()
    print(f"context init {init_s * 1e3:.0f} ms, key material {kb / 1e6:.1f} MB")
    if 1 not in T.available_kernels():      # product build
        assert kb < 185e6, kb


def test_keyswitch_v4_layout_subprocess():
    """TFHE_AMD_KS5=0 (read once per process) builds the ks-v4 layout instead of the MFMA key
    switch's: that path, key-index split (<= 768) and plain, still equals the oracle."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np
sys.path[:0] = [%r, %r]
import tfhe_amd as T, oracle_ctypes as O
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); o = O.OracleKey(K.bk, K.ksk)
rng = np.random.default_rng(3)
for B in (400, 769):
    u_a = rng.integers(-2**31, 2**31, (B, 1024), dtype=np.int64).astype(np.int32)
    u_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    k_a, k_b = c.keyswitch_host(u_a, u_b); o_a, o_b = o.keyswitch_batch(u_a, u_b)
    assert np.array_equal(k_a, o_a) and np.array_equal(k_b, o_b), B
print("ks-v4 ok", c.key_bytes())
""" % (os.path.join(REPO, "cpu-gpu-tfhe_amd"), os.path.join(REPO, "tests"))
    env = dict(os.environ, TFHE_AMD_KS5="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ks-v4 ok" in r.stdout


def test_register_rotation_subprocess():
    """TFHE_AMD_V6_RREG=1 (read once per process) forces the register / ds_bpermute rotation of
    cmux_v6 — the default only above one workgroup per CU — onto small launches: the CMux steps
    at the rotation edges (a = 0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048), every register
    shift q = a >> 6 of the throughput kernels' 32-way permutation, and woKS with bara = 0 runs
    still equal the oracle."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path[:0] = [%r, %r]
import tfhe_amd as T, oracle_ctypes as O
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); o = O.OracleKey(K.bk, K.ksk)
rng = np.random.default_rng(5)
B, iters = 4, 32
acc0 = rng.integers(-2**31, 2**31, (B, 2, 1024), dtype=np.int64).astype(np.int32)
bara = rng.integers(0, 2049, (B, iters), dtype=np.int64).astype(np.int32)
bara[0, :10] = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048]
bara[1, :10] = [127, 128, 129, 960, 1087, 1088, 1984, 2000, 31, 32]
q = np.arange(32)
bara[2] = 64 * q + np.mod(7 * q, 64)     # every register shift q with assorted lane shifts
bara[3] = 64 * q + 63 - q
d_acc = torch.from_numpy(acc0.copy()).cuda()
c.blind_rotate_dev(d_acc, torch.from_numpy(bara).cuda(), iters); c.sync()
got = d_acc.cpu().numpy()
for b in range(B):
    want = acc0[b].copy()
    for i in range(iters):
        if bara[b, i] != 0:
            want = o.mux_rotate(want, i, int(bara[b, i]))
    assert np.array_equal(got[b], want), b
x_a = rng.integers(-2**31, 2**31, (8, 500), dtype=np.int64).astype(np.int32)
x_b = rng.integers(-2**31, 2**31, 8, dtype=np.int64).astype(np.int32)
x_a[1, :50] = 0
u = c.woks_host(T.MU, x_a, x_b); w = o.woks_batch(T.MU, x_a, x_b)
assert np.array_equal(u[0], w[0]) and np.array_equal(u[1], w[1])
print("rreg ok")
""" % (os.path.join(REPO, "cpu-gpu-tfhe_amd"), os.path.join(REPO, "tests"))
    env = dict(os.environ, TFHE_AMD_V6_RREG="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rreg ok" in r.stdout


def test_paired_barrier_variant_subprocess():
    """TFHE_AMD_V6P_PAIRSYNC=0 (read once per process) runs the paired kernel with the workgroup
    barrier instead of the per-ciphertext LDS counters: a 301-gate batch (an odd count, so one
    padding ciphertext) and a 199-gate MUX batch equal the oracle."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path[:0] = [%r, %r]
import tfhe_amd as T, oracle_ctypes as O
K = T.SecretKeyset(); c = T.Context(K.bk, K.ksk, device=0); o = O.OracleKey(K.bk, K.ksk)
rng = np.random.default_rng(6)
x, y = rng.integers(0, 2, 301), rng.integers(0, 2, 301)
(a_a, a_b), (b_a, b_b) = K.encrypt(x, rng), K.encrypt(y, rng)
r = c.gate_host("NAND", a_a, a_b, b_a, b_b)
kern = c.last_kernels()
w = o.gate_batch("NAND", a_a, a_b, b_a, b_b)
assert np.array_equal(r[0], w[0]) and np.array_equal(r[1], w[1])   # parity first, then which kernel
assert any("v6p(paired+reg-rotation)" in k for k in kern), kern
s, x, y = (rng.integers(0, 2, 199) for _ in range(3))
(sa, sb), (xa, xb), (ya, yb) = (K.encrypt(v, rng) for v in (s, x, y))
r = c.gate_host("MUX", sa, sb, xa, xb, ya, yb); w = o.gate_batch("MUX", sa, sb, xa, xb, ya, yb)
assert np.array_equal(r[0], w[0]) and np.array_equal(r[1], w[1])
print("barrier ok")
""" % (os.path.join(REPO, "cpu-gpu-tfhe_amd"), os.path.join(REPO, "tests"))
    env = dict(os.environ, TFHE_AMD_V6P_PAIRSYNC="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "barrier ok" in r.stdout


def test_fp64_ceiling_measurement():
    """tfhe_amd_fp64_ceiling (bench.py's roofline.sustained): a plausible fp64 rate and clock, and
    the caller's current device left as it was."""
    torch = _torch()
    dev = torch.cuda.current_device()
    tf, mhz = T.fp64_ceiling(0, 2, 0.2)
    assert 10.0 < tf < 80.0, tf          # MI355X fp64 vector peak 78.6 TFLOP/s
    assert 500.0 < mhz < 2600.0, mhz
    assert torch.cuda.current_device() == dev
    with pytest.raises(T.TfheAmdError):
        T.fp64_ceiling(0, 0, 1.0)


@pytest.mark.gpu
def test_mixed_gate_batch_bit_exact(ctx, okey, keyset, rng):
    """tfhe_amd_gate_batch_mixed_host: all 11 gate kinds interleaved in one batch (one blind
    rotation over 1 row per gate, 2 per MUX, one key switch) — every output equals the oracle's
    gate of its kind word for word, for a small batch (one row per CU) and one above a round of
    rows per CU (300 gates, ~330 rows: the register-rotation kernel), and decrypts right."""
    names = ["NAND", "OR", "AND", "XOR", "XNOR", "NOR", "ANDNY", "ANDYN", "ORNY", "ORYN", "MUX"]
    truth = {"NAND": lambda a, b, c: 1 - (a & b), "OR": lambda a, b, c: a | b, "AND": lambda a, b, c: a & b,
             "XOR": lambda a, b, c: a ^ b, "XNOR": lambda a, b, c: 1 - (a ^ b), "NOR": lambda a, b, c: 1 - (a | b),
             "ANDNY": lambda a, b, c: (1 - a) & b, "ANDYN": lambda a, b, c: a & (1 - b),
             "ORNY": lambda a, b, c: (1 - a) | b, "ORYN": lambda a, b, c: a | (1 - b),
             "MUX": lambda a, b, c: np.where(a == 1, b, c)}
    for B in (37, 300):
        gates = [names[i % len(names)] if i % 7 else names[rng.integers(0, len(names))] for i in range(B)]
        xa, xb, xc = (rng.integers(0, 2, B) for _ in range(3))
        (aa, ab), (ba, bb), (ca, cb) = (keyset.encrypt(v, rng) for v in (xa, xb, xc))
        r_a, r_b = ctx.gate_mixed_host(gates, aa, ab, ba, bb, ca, cb)
        kern = ",".join(ctx.last_kernels())
        g = np.array(gates)
        for name in names:
            idx = np.flatnonzero(g == name)
            if idx.size == 0:
                continue
            args = [aa[idx], ab[idx], ba[idx], bb[idx]] + ([ca[idx], cb[idx]] if name == "MUX" else [])
            o_a, o_b = okey.gate_batch(name, *args)
            assert np.array_equal(r_a[idx], o_a) and np.array_equal(r_b[idx], o_b), (B, name)
            want = truth[name](xa[idx], xb[idx], xc[idx])
            assert np.array_equal(keyset.decrypt(r_a[idx], r_b[idx]), want), (B, name)
        assert "k_blind_rotate_v6_rows" in kern, kern   # parity first, then which kernel
