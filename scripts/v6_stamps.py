"""Phase timing of the v6 blind rotation (dev tool): run with TFHE_AMD_LIB pointing at a
-DTFHE_AMD_V6_STAMPS build; prints average shader-clock cycles per CMux step per phase of the
two waves of workgroup 0 while a batch of B ciphertexts runs (B from argv, default 1024)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-gpu-tfhe_amd"))
import tfhe_amd as T  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
T.select_kernel(6)
K = T.SecretKeyset()
ctx = T.Context(K.bk, K.ksk, device=0)
rng = np.random.default_rng(1)
x = rng.integers(0, 2, B)
a_a, a_b = K.encrypt(x, rng)
ctx.gate_host("NAND", a_a, a_b, a_a, a_b)
buf = (ctypes.c_ulonglong * 24)()
T.lib.tfhe_amd_debug_v6_stamps(buf, 1)
ctx.gate_host("NAND", a_a, a_b, a_a, a_b)
T.lib.tfhe_amd_debug_v6_stamps(buf, 0)
names = ["ext+decomp", "fwd A,B", "passC+mac1", "mac2", "barrier1", "add+invC", "barrier2", "inv B,A",
         "acc update", "loop"]
for wv in (0, 1):
    tot = sum(buf[wv * 12 + k] for k in range(10))
    print(f"B={B} wave {wv}: total cycles/step {tot / 500:.0f}")
    for k, n in enumerate(names):
        print(f"  {n:12s} {buf[wv * 12 + k] / 500:8.0f}")
