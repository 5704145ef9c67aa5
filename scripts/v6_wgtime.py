"""Per-workgroup time windows of the v6 blind rotation (dev tool): run with TFHE_AMD_LIB pointing
at a -DTFHE_AMD_V6_STAMPS build.  Prints how the launch's wall time splits into workgroup
lifetimes: start skew, duration spread, shader clock per workgroup, grouping by XCC / CU."""
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
for _ in range(3):
    ctx.gate_host("NAND", a_a, a_b, a_a, a_b)
n = min(B, 8192)
buf = (ctypes.c_ulonglong * (n * 6))()
T.lib.tfhe_amd_debug_v6_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert T.lib.tfhe_amd_debug_v6_wgtime(buf, n) == 0
d = np.frombuffer(buf, dtype=np.uint64).reshape(n, 6).astype(np.int64)
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/wgtime_{B}{os.environ.get('WG_TAG', '')}.npy", d)
t0 = d[:, 0].min()
st = (d[:, 0] - t0) * 10.0 / 1000      # us (100 MHz)
en = (d[:, 1] - t0) * 10.0 / 1000
dur = en - st
clk = (d[:, 3] - d[:, 2]) / np.maximum(dur, 1e-9) / 1000   # GHz
hw = d[:, 4]
xcc = d[:, 5] & 0xF
cu = (hw >> 8) & 0xF
sh_ = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
print(f"B={B}: launch window {en.max():.0f} us; start skew max {st.max():.1f} us")
print(f"  duration us: min {dur.min():.0f} p10 {np.percentile(dur,10):.0f} med {np.median(dur):.0f} p90 {np.percentile(dur,90):.0f} max {dur.max():.0f}")
print(f"  clock GHz: min {clk.min():.3f} med {np.median(clk):.3f} max {clk.max():.3f}")
key = xcc * 1000 + se * 100 + sh_ * 16 + cu
ucu, cnt = np.unique(key, return_counts=True)
print(f"  distinct CUs used {len(ucu)}; workgroups per CU histogram:", dict(zip(*np.unique(cnt, return_counts=True))))
per_cu_dur = {k: dur[key == k].mean() for k in ucu}
for c in sorted(set(cnt)):
    ks = [k for k, m in zip(ucu, cnt) if m == c]
    print(f"    CUs with {c} WGs: mean WG duration {np.mean([per_cu_dur[k] for k in ks]):.0f} us")
rank = np.arange(n) // 256     # dispatch rank on the CU (256 CUs: b, b+256, ... share one)
for r_ in range(int(rank.max()) + 1 if n <= 1024 else 0):
    m = rank == r_
    print(f"  rank {r_}: dur med {np.median(dur[m]):.0f} p90 {np.percentile(dur[m], 90):.0f} max {dur[m].max():.0f}")
print(f"  launch / mean duration {en.max() / dur.mean():.3f}")
for x_ in range(8):
    m = xcc == x_
    if m.any():
        print(f"  xcc {x_}: {m.sum()} WGs, dur med {np.median(dur[m]):.0f} max {dur[m].max():.0f}, end max {en[m].max():.0f}")
