"""The optimized CPU baseline (oracle/cpu_fft.c: fp64 FFT external product, OpenMP over gates;
bench.py's cpu_baseline leg) is Torus32-identical to the exact oracle, so the GPU/CPU ratio
compares the same computation.  CPU only."""
import numpy as np
import pytest

import oracle_ctypes as O


@pytest.fixture(scope="module")
def fkey(keyset):
    return O.CpuFftKey(keyset.bk, keyset.ksk)


@pytest.mark.parametrize("gate", ["NAND", "XOR", "ANDNY"])
def test_cpu_fft_gates_match_oracle(fkey, okey, keyset, rng, gate):
    B = 6
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = keyset.encrypt(x, rng), keyset.encrypt(y, rng)
    got = fkey.gate_batch(gate, a_a, a_b, b_a, b_b, nthreads=4)
    want = okey.gate_batch(gate, a_a, a_b, b_a, b_b, nthreads=4)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert fkey.max_round_error() < 0.25


def test_cpu_fft_woks_edges_match_oracle(fkey, okey, rng):
    """woKS on random LWE inputs with the modswitch wrap edge and skipped CMux steps."""
    B = 4
    x_a = rng.integers(-2**31, 2**31, (B, 500), dtype=np.int64).astype(np.int32)
    x_b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
    x_b[0] = np.int32(-2**20 + 5)
    x_a[1, :50] = 0
    got = fkey.woks_batch(1 << 29, x_a, x_b, nthreads=4)
    want = okey.woks_batch(1 << 29, x_a, x_b, nthreads=4)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
