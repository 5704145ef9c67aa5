"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"`: oracle vs golden fixtures, host logic, C-ABI load/exports (no GPU).
`-m gpu`: parity of the HIP path (through the C ABI) against the CPU oracle.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cpu-gpu-tfhe_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def keyset():
    import tfhe_amd as T
    K = T.SecretKeyset()
    yield K
    K.close()


@pytest.fixture(scope="session")
def okey(keyset):
    import oracle_ctypes as O
    return O.OracleKey(keyset.bk, keyset.ksk, use_ntt=True)


@pytest.fixture(scope="session")
def ctx(keyset):
    import tfhe_amd as T
    c = T.Context(keyset.bk, keyset.ksk, device=0)
    yield c
    c.close()


@pytest.fixture
def rng(request):
    return np.random.default_rng(abs(hash(request.node.name)) % (2**32))
