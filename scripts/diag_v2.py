"""GPU diagnostic: v2 vs v1 vs oracle on single CMux steps; prints mismatch structure."""
import sys, os
import numpy as np
sys.path.insert(0, "cpu-gpu-tfhe_amd"); sys.path.insert(0, "tests")
import tfhe_amd as T, oracle_ctypes as O
import torch
K = T.SecretKeyset()
ctx = T.Context(K.bk, K.ksk)
ok = O.OracleKey(K.bk, K.ksk, use_ntt=True)
rng = np.random.default_rng(3)
for B in (1, 2, 8):
    for ver in (1, 2):
        T.lib.tfhe_amd_select_kernel(ver)
        for a in (1, 77, 1024, 1500):
            acc0 = rng.integers(-2**31, 2**31, (B, 2, 1024), dtype=np.int64).astype(np.int32)
            bara = np.full((B, 1), a, np.int32)
            d = torch.from_numpy(acc0.copy()).cuda()
            ctx.blind_rotate_dev(d, torch.from_numpy(bara).cuda(), 1)
            ctx.sync()
            got = d.cpu().numpy()
            bad = []
            for b in range(B):
                want = ok.mux_rotate(acc0[b], 0, a)
                diff = got[b] != want
                bad.append(int(diff.sum()))
                if b == 0 and diff.any():
                    js = np.nonzero(diff)
                    c, j = js[0], js[1]
                    L = j % 64; r = j // 64
                    print(f"   B={B} v{ver} a={a}: c-hist {np.bincount(c, minlength=2)} r-hist {np.bincount(r, minlength=16)} "
                          f"L-hist(first 16) {np.bincount(L, minlength=64)[:16]}")
            print(f"B={B} v{ver} a={a}: mismatches per ct {bad}", flush=True)
