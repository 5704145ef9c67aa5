"""Dev tool (GPU box): does recording the engine's per-launch HIP events (bench.py's kernel timing,
tfhe_amd_profile_enable) slow the timed steps?  Alternates K-step runs with and without them."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-gpu-tfhe_amd"))
import tfhe_amd as T  # noqa: E402

B, K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 20
Ks = T.SecretKeyset()
ctx = T.Context(Ks.bk, Ks.ksk, device=0)
rng = np.random.default_rng(1)
x = rng.integers(0, 2, B)
a_a, a_b = Ks.encrypt(x, rng)
dev = [torch.from_numpy(v).cuda() for v in (a_a, a_b, a_a, a_b)]
r_a = torch.empty((B, 500), dtype=torch.int32, device="cuda")
r_b = torch.empty(B, dtype=torch.int32, device="cuda")
ctx.reserve(B)
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    ctx.gate_dev("NAND", r_a, r_b, *dev, stream=s)
torch.cuda.synchronize()
for rep in range(3):
    for prof in (False, True):
        if prof:
            ctx.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(K):
            ctx.gate_dev("NAND", r_a, r_b, *dev, stream=s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        extra = ""
        if prof:
            p = ctx.profile_read()
            ctx.profile_enable(False)
            extra = " br %.3f ks %.3f" % (p["br_ms"] / p["br_launches"], p["ks_ms"] / p["ks_launches"])
        print("B=%d events=%d  %.4f ms/step%s" % (B, prof, ms, extra), flush=True)
