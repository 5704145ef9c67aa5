"""Batched circuit schedules: csrc/circuit.cpp.

CPU: the builders (ripple / prefix adders, subtractor, Dadda multiplier, MUX, NOT / CONST
folding, threshold rows) are evaluated in plaintext through `Circuit.eval_plain`, which uses
the same +-1/8 torus encodings and sign rule as the GPU rows, against integer arithmetic
(reference semantics: Cipher.cpp operator+ / operator- / operator*, main.cu:1483-1579).
GPU: the same circuits run level by level on the MI355X; decryptions must equal the
plaintext results for every instance."""
import numpy as np
import pytest

import tfhe_amd as T


def _bits(wires, x, n):
    return dict(zip(wires, T.bits_of(x, n)))


def _value(val, wires):
    return T.int_of([val[w] for w in wires])


@pytest.mark.parametrize("n", [1, 4, 16, 32])
def test_ripple_adder_plain(n, rng):
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    s, co = C.add(a, b)
    info = C.info()
    assert info["depth"] == n and info["bootstraps"] == 2 * n
    x = rng.integers(0, 2**n, 200)
    y = rng.integers(0, 2**n, 200)
    x[:2] = [0, 2**n - 1]
    y[:2] = [0, 2**n - 1]
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    assert np.array_equal(_value(val, s + [co]), x + y)


@pytest.mark.parametrize("n", [2, 8, 32])
def test_prefix_adder_plain(n, rng):
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    s, co = C.add_prefix(a, b)
    assert C.info()["depth"] <= 2 + int(np.ceil(np.log2(n)))
    x = rng.integers(0, 2**n, 300)
    y = rng.integers(0, 2**n, 300)
    x[:3] = [2**n - 1, 2**n - 1, 0]
    y[:3] = [1, 2**n - 1, 0]
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    assert np.array_equal(_value(val, s + [co]), x + y)


@pytest.mark.parametrize("n", [4, 16])
def test_subtractor_plain(n, rng):
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    d, _ = C.sub(a, b)
    x = rng.integers(0, 2**n, 200)
    y = rng.integers(0, 2**n, 200)
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    assert np.array_equal(_value(val, d), (x - y) % 2**n)
    # NOT and CONST are folded: no bootstraps beyond the 2 per bit of the adder
    assert C.info()["bootstraps"] == 2 * n


@pytest.mark.parametrize("n", [1, 3, 8, 16])
def test_multiplier_plain(n, rng):
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    p = C.mul(a, b)
    x = rng.integers(0, 2**n, 200)
    y = rng.integers(0, 2**n, 200)
    x[:2] = [2**n - 1, 0]
    y[:2] = [2**n - 1, 2**n - 1]
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    assert np.array_equal(_value(val, p), x * y)
    if n == 16:
        assert C.info()["depth"] <= 14


def test_mux_and_gates_plain(rng):
    C = T.Circuit()
    a, b, c = C.inputs(3)
    outs = {name: C.gate(name, a, b) for name in
            ("NAND", "OR", "AND", "XOR", "XNOR", "NOR", "ANDNY", "ANDYN", "ORNY", "ORYN")}
    outs["MUX"] = C.gate("MUX", a, b, c)
    outs["MAJ"] = C.gate("MAJ", a, b, c)
    outs["XOR3"] = C.gate("XOR3", a, b, c)
    nb = C.gate("NOT", b)
    outs["AND_NOTB"] = C.gate("AND", a, nb)
    outs["CONST1_XOR"] = C.gate("XOR", a, C.gate("CONST", 1))
    x, y, z = (rng.integers(0, 2, 64) for _ in range(3))
    val = C.eval_plain({a: x, b: y, c: z})
    want = {"NAND": 1 - (x & y), "OR": x | y, "AND": x & y, "XOR": x ^ y, "XNOR": 1 - (x ^ y),
            "NOR": 1 - (x | y), "ANDNY": (1 - x) & y, "ANDYN": x & (1 - y), "ORNY": (1 - x) | y,
            "ORYN": x | (1 - y), "MUX": np.where(x == 1, y, z), "MAJ": (x + y + z >= 2).astype(int),
            "XOR3": x ^ y ^ z, "AND_NOTB": x & (1 - y), "CONST1_XOR": 1 - x}
    for k, w in outs.items():
        assert np.array_equal(val[w], want[k]), k


def test_builder_errors():
    C = T.Circuit()
    a = C.inputs(2)
    with pytest.raises(T.TfheAmdError):
        C.gate("AND", a[0], 99)          # undefined wire
    with pytest.raises(T.TfheAmdError):
        C.gate(77, a[0], a[1])           # unknown gate
    with pytest.raises(T.TfheAmdError):
        C.gate("MUX", a[0], a[1])        # missing third input


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_circuit_gates_gpu(ctx, keyset, rng):
    C = T.Circuit()
    a, b, c = C.inputs(3)
    names = ("NAND", "XOR", "ANDNY", "MUX", "MAJ", "XOR3")
    outs = {k: (C.gate(k, a, b, c) if k in ("MUX", "MAJ", "XOR3") else C.gate(k, a, b)) for k in names}
    nb = C.gate("NOT", b)
    outs["NOTB"] = nb
    outs["OR_NOTB"] = C.gate("OR", a, nb)
    B = 96
    x, y, z = (rng.integers(0, 2, B) for _ in range(3))
    got = C.run(ctx, B, {a: x, b: y, c: z}, list(outs.values()), keyset, rng)
    want = C.eval_plain({a: x, b: y, c: z})
    for k, w in outs.items():
        assert np.array_equal(got[w], want[w]), k


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ripple", "prefix", "sub"])
def test_adders_gpu(ctx, keyset, rng, kind):
    n, B = 16, 64
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    if kind == "ripple":
        s, co = C.add(a, b)
        outs, want_f = s + [co], (lambda x, y: x + y)
    elif kind == "prefix":
        s, co = C.add_prefix(a, b)
        outs, want_f = s + [co], (lambda x, y: x + y)
    else:
        s, _ = C.sub(a, b)
        outs, want_f = s, (lambda x, y: (x - y) % 2**n)
    x = rng.integers(0, 2**n, B)
    y = rng.integers(0, 2**n, B)
    got = C.run(ctx, B, {**_bits(a, x, n), **_bits(b, y, n)}, outs, keyset, rng)
    assert np.array_equal(_value(got, outs), want_f(x, y))


@pytest.mark.gpu
def test_multiplier_gpu(ctx, keyset, rng):
    n, B = 8, 32
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    p = C.mul(a, b)
    x = rng.integers(0, 2**n, B)
    y = rng.integers(0, 2**n, B)
    got = C.run(ctx, B, {**_bits(a, x, n), **_bits(b, y, n)}, p, keyset, rng)
    assert np.array_equal(_value(got, p), x * y)


@pytest.mark.gpu
def test_noise_margins_gpu(ctx, keyset, rng):
    """Phase noise of bootstrapped + key-switched outputs, and the decision margin it leaves
    for the circuit rows that sum 3 of them (MAJ, XOR3 at weight 2, the prefix adder's
    2/1/1 threshold row).  Margins in standard deviations of the summed input noise."""
    B = 4096
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a_a, a_b = keyset.encrypt(x, rng)
    b_a, b_b = keyset.encrypt(y, rng)
    r_a, r_b = ctx.gate_host("NAND", a_a, a_b, b_a, b_b)
    ph = keyset.phase(r_a, r_b).astype(np.int64)
    want = np.where((1 - (x & y)) == 1, 1 << 29, -(1 << 29))
    err = (ph - want) / 2.0**32
    sigma = float(np.std(err))
    assert np.all(np.abs(err) < 1 / 16), float(np.max(np.abs(err)))
    margins = {"NAND": (1 / 8) / (np.sqrt(2) * sigma), "MAJ": (1 / 8) / (np.sqrt(3) * sigma),
               "XOR3": (1 / 4) / (2 * np.sqrt(3) * sigma), "THRESH_2_1_1": (1 / 8) / (np.sqrt(6) * sigma)}
    print(f"bootstrapped output noise sigma = 2^{np.log2(sigma):.2f}; margins (sigmas): "
          + ", ".join(f"{k} {v:.1f}" for k, v in margins.items()))
    assert min(margins.values()) > 6.0


# ---------------------------------------------------------------- Cipher's remaining operators

def _signed(v, n):
    v = np.asarray(v, dtype=np.int64) & (2**n - 1)
    return np.where(v >= 2**(n - 1), v - 2**n, v)


CMP_F = {"GT": np.greater, "GE": np.greater_equal, "LT": np.less, "LE": np.less_equal,
         "EQ": np.equal, "NE": np.not_equal}


def _cmp_inputs(rng, n, k=300):
    x = rng.integers(0, 2**n, k)
    y = rng.integers(0, 2**n, k)
    e, l1, m1 = k // 5, 3 * k // 10, 2 * k // 5
    y[:e] = x[:e]                                     # equal pairs
    y[e:l1] = x[e:l1] ^ 1                             # differ in the lsb only
    y[l1:m1] = x[l1:m1] ^ (1 << (n - 1))              # differ in the msb only
    x[m1:m1 + 2] = [0, 2**n - 1]
    y[m1:m1 + 2] = [2**n - 1, 0]
    return x, y


@pytest.mark.parametrize("n", [1, 3, 8, 16])
@pytest.mark.parametrize("signed", [False, True])
def test_compare_plain(n, signed, rng):
    """operator> / <= / == (Cipher.cpp:597-644) and the other three, unsigned and two's
    complement, as log-depth circuits."""
    if signed and n == 1:
        pytest.skip("a 1-bit two's complement integer is only a sign")
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    outs = {op: C.compare(a, b, op, signed) for op in CMP_F}
    x, y = _cmp_inputs(rng, n)
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    xv, yv = (_signed(x, n), _signed(y, n)) if signed else (x, y)
    for op, w in outs.items():
        assert np.array_equal(val[w], CMP_F[op](xv, yv).astype(int)), op
    if n == 16:
        assert C.info()["depth"] <= 2 + int(np.ceil(np.log2(n))) + 1


@pytest.mark.parametrize("n", [4, 16])
@pytest.mark.parametrize("signed", [False, True])
def test_minmax_plain(n, signed, rng):
    """minimum (Cipher.cpp:314-333, unsigned) and max, also two's complement."""
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    lo, hi = C.minmax(a, b, False, signed), C.minmax(a, b, True, signed)
    x, y = _cmp_inputs(rng, n)
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    xv, yv = (_signed(x, n), _signed(y, n)) if signed else (x, y)
    got_lo, got_hi = _value(val, lo), _value(val, hi)
    if signed:
        got_lo, got_hi = _signed(got_lo, n), _signed(got_hi, n)
    assert np.array_equal(got_lo, np.minimum(xv, yv)) and np.array_equal(got_hi, np.maximum(xv, yv))


@pytest.mark.parametrize("n", [2, 8, 16])
def test_neg_abs_plain(n, rng):
    """twosComplement (Cipher.cpp:300-311) and absolute (:483-505), two's complement mod 2^n."""
    C = T.Circuit()
    a = C.inputs(n)
    ng, ab = C.neg(a), C.abs(a)
    x = rng.integers(0, 2**n, 300)
    x[:4] = [0, 1, 2**(n - 1), 2**n - 1]
    val = C.eval_plain(_bits(a, x, n))
    xs = _signed(x, n)
    assert np.array_equal(_value(val, ng), (-xs) % 2**n)
    assert np.array_equal(_value(val, ab), np.abs(xs) % 2**n)


@pytest.mark.parametrize("n", [1, 4, 8])
def test_divu_plain(n, rng):
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    q, r = C.divu(a, b)
    x = rng.integers(0, 2**n, 300)
    y = rng.integers(1, 2**n, 300)
    x[:3] = [2**n - 1, 0, 2**n - 1]
    y[:3] = [1, 1, 2**n - 1]
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    assert np.array_equal(_value(val, q), x // y) and np.array_equal(_value(val, r), x % y)


@pytest.mark.parametrize("n", [4, 8, 16])
def test_signed_div_plain(n, rng):
    """operator/ (Cipher.cpp:507-589): |a| / |b| by restoring division, negated when the signs
    differ: truncation toward zero, mod 2^n."""
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    q = C.div(a, b)
    x = rng.integers(0, 2**n, 200)
    y = rng.integers(0, 2**n, 200)
    y[y == 0] = 1
    x[:4] = [2**(n - 1), 2**(n - 1), 2**n - 1, 5 % 2**n]       # -2^(n-1) / -1 wraps
    y[:4] = [2**n - 1, 1, 2**n - 1, 2**n - 3 if n > 2 else 1]
    val = C.eval_plain({**_bits(a, x, n), **_bits(b, y, n)})
    xs, ys = _signed(x, n), _signed(y, n)
    want = np.array([(-1 if (p < 0) != (d < 0) else 1) * (abs(int(p)) // abs(int(d))) for p, d in zip(xs, ys)])
    assert np.array_equal(_value(val, q), want % 2**n)


@pytest.mark.gpu
def test_cipher_operators_gpu(ctx, keyset, rng):
    """The new builders on the MI355X, 16-bit operands, 48 instances per launch: signed >,
    unsigned ==, minimum, absolute and signed division decrypt to the integer results."""
    n, B = 16, 48
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    gt = C.compare(a, b, "GT", True)
    eq = C.compare(a, b, "EQ")
    mn = C.minmax(a, b)
    ab = C.abs(a)
    x, y = _cmp_inputs(rng, n, B)
    outs = [gt, eq] + mn + ab
    got = C.run(ctx, B, {**_bits(a, x, n), **_bits(b, y, n)}, outs, keyset, rng)
    xs, ys = _signed(x, n), _signed(y, n)
    assert np.array_equal(got[gt], (xs > ys).astype(int))
    assert np.array_equal(got[eq], (x == y).astype(int))
    assert np.array_equal(_value(got, mn), np.minimum(x, y))
    assert np.array_equal(_value(got, ab), np.abs(xs) % 2**n)


@pytest.mark.gpu
def test_signed_division_gpu(ctx, keyset, rng):
    n, B = 8, 32
    C = T.Circuit()
    a, b = C.inputs(n), C.inputs(n)
    q = C.div(a, b)
    x = rng.integers(0, 2**n, B)
    y = rng.integers(1, 2**n, B)
    got = C.run(ctx, B, {**_bits(a, x, n), **_bits(b, y, n)}, q, keyset, rng)
    xs, ys = _signed(x, n), _signed(y, n)
    want = np.array([(-1 if (p < 0) != (d < 0) else 1) * (abs(int(p)) // abs(int(d))) for p, d in zip(xs, ys)])
    assert np.array_equal(_value(got, q), want % 2**n)
    print(f"8-bit signed division circuit: depth {C.info()['depth']}, {C.info()['bootstraps']} bootstraps")


def test_circuit_oracle_evaluator_decrypts_like_plaintext(keyset, okey):
    """The checker of tests/test_configs_gpu.py::test_circuits_every_wire_torus32_vs_oracle
    (tests/circuit_oracle.py, exact oracle bootstraps node by node) decrypts, on every wire of a
    small circuit with NOT / CONST / MUX / MAJ / XOR3 / lincomb nodes, to the circuit's plaintext
    evaluation (CPU only)."""
    import circuit_oracle
    rng = np.random.default_rng(3)
    C = T.Circuit()
    a, b = C.inputs(3), C.inputs(3)
    s, co = C.add(a, b)
    mn = C.minmax(a, b)
    na = C.gate("NOT", a[0])
    one = C.gate("CONST", 1)
    C.gate("MUX", na, one, b[1])
    C.lincomb(1 << 29, 2, a[1], 1, b[2], 1, na)
    B = 2
    bits = {w: rng.integers(0, 2, B) for w in a + b}
    enc = {w: keyset.encrypt(v, rng) for w, v in bits.items()}
    W = circuit_oracle.eval_circuit(C, okey, enc, B, nthreads=8)
    ref = C.eval_plain(bits)
    for w in range(C.info()["wires"]):
        dec = keyset.decrypt(*W[w])
        assert np.array_equal(dec, np.broadcast_to(ref[w], dec.shape)), w   # CONST wires: a scalar


@pytest.mark.gpu
def test_circuit_state_dropped_with_its_context(keyset, rng):
    """A circuit keeps device state (level tables, scratch) per executing context; destroying the
    context drops it (keyed by a never-reused context uid, so a context allocated later at the
    same address starts clean).  One circuit on 4 successive contexts: at most one state at a
    time, none after each context is closed, results right every time."""
    import torch
    C = T.Circuit()
    a, b = C.inputs(2)
    o = C.gate("XOR", a, b)
    B = 8
    free0 = None
    for k in range(4):
        c = T.Context(keyset.bk, keyset.ksk, device=0)
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        got = C.run(c, B, {a: x, b: y}, [o], keyset, rng)
        assert np.array_equal(got[o], x ^ y)
        assert C.state_count() == 1
        c.close()
        assert C.state_count() == 0
        torch.cuda.synchronize()
        free = torch.cuda.mem_get_info()[0]
        if free0 is None:
            free0 = free
        assert abs(free - free0) < (64 << 20), "device memory grows with each context"
    C.close()
