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
