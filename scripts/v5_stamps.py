"""Phase timing of the v5 latency kernel (dev tool): run with TFHE_AMD_LIB pointing at a
-DTFHE_AMD_V5_STAMPS build; prints average shader-clock cycles per CMux step per phase."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-gpu-tfhe_amd"))
import tfhe_amd as T  # noqa: E402

T.select_kernel(5)
K = T.SecretKeyset()
ctx = T.Context(K.bk, K.ksk, device=0)
rng = np.random.default_rng(1)
x = rng.integers(0, 2, 1)
a_a, a_b = K.encrypt(x, rng)
ctx.gate_host("NAND", a_a, a_b, a_a, a_b)
buf = (ctypes.c_ulonglong * 24)()
T.lib.tfhe_amd_debug_v5_stamps(buf, 1)
ctx.gate_host("NAND", a_a, a_b, a_a, a_b)
T.lib.tfhe_amd_debug_v5_stamps(buf, 0)
names = ["decomp", "fwd+storeC", "B1", "MAC", "B1b", "inverse", "twist+give", "B2", "take", "B3"]
for wv, label in ((0, "MAC wave 0"), (1, "idle wave 2")):
    tot = sum(buf[wv * 12 + k] for k in range(10))
    print(label, "total cycles/step %.0f" % (tot / 500))
    for k, n in enumerate(names):
        print(f"  {n:12s} {buf[wv * 12 + k] / 500:8.0f}")
