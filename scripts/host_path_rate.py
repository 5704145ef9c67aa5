"""PCIe-inclusive rate of the host-pointer batch API (tfhe_amd_gate_batch_host): inputs in host
memory, staged through pinned buffers, one H2D, the device batch, one D2H, results back in host
memory.  Prints one JSON line per batch size (DESIGN.md §6 quotes it next to bench.py's
HBM-resident value)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-gpu-tfhe_amd"))
import tfhe_amd as T  # noqa: E402

PINNED = os.environ.get("HOST_PATH_PINNED", "0") == "1"   # caller-owned pinned arrays (T.host_copy)
K = T.SecretKeyset()
ctx = T.Context(K.bk, K.ksk, device=0)
rng = np.random.default_rng(5)
for B in [int(b) for b in (sys.argv[1:] or ["1", "1024", "4096"])]:
    x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
    (a_a, a_b), (b_a, b_b) = K.encrypt(x, rng), K.encrypt(y, rng)
    ctx.reserve(B)
    # results into reused, already-touched arrays (a C caller's buffers): fresh numpy arrays would
    # add the first-touch page faults of B x 2 KB to every call
    out = (np.zeros((B, 500), np.int32), np.zeros(B, np.int32))
    if PINNED:
        a_a, a_b, b_a, b_b = (T.host_copy(v) for v in (a_a, a_b, b_a, b_b))
        out = (T.host_empty((B, 500)), T.host_empty(B))
    for _ in range(2):
        r_a, r_b = ctx.gate_host("NAND", a_a, a_b, b_a, b_b, out=out)
    reps = 15
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r_a, r_b = ctx.gate_host("NAND", a_a, a_b, b_a, b_b, out=out)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))   # median call: a shared box's scheduling hiccups stay out of it
    ok = bool(np.array_equal(K.decrypt(r_a, r_b), 1 - (x & y)))
    # the same batch from HBM-resident inputs (device API), same process, for the overhead
    import torch
    dev = [torch.from_numpy(v).cuda() for v in (a_a, a_b, b_a, b_b)]
    d_a = torch.empty((B, 500), dtype=torch.int32, device="cuda")
    d_b = torch.empty(B, dtype=torch.int32, device="cuda")
    ctx.gate_dev("NAND", d_a, d_b, *dev)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.gate_dev("NAND", d_a, d_b, *dev)
    ctx.sync()
    dd = (time.perf_counter() - t0) / reps
    # the same device batch called synchronously (synchronize after each call, as the host path's
    # own synchronous contract does): the device-side part of a synchronous call's cost
    tsync = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.gate_dev("NAND", d_a, d_b, *dev)
        ctx.sync()
        tsync.append(time.perf_counter() - t0)
    ds = float(np.median(tsync))
    print(json.dumps({"batch": B, "ms_per_call": dt * 1e3, "ms_min": min(ts) * 1e3, "ms_mean": float(np.mean(ts)) * 1e3,
                      "statistic": "median of %d calls" % reps, "gate_bootstraps_per_s": B / dt, "truth_table_ok": ok,
                      "device_path_ms": dd * 1e3, "device_path_sync_ms": ds * 1e3, "slice": 1024,
                      "path": "host pointers, caller-owned pinned arrays (DMA straight from and into them)" if PINNED
                      else "host pointers (pinned staging + PCIe both ways)", "engine": T.version()}))
ctx.close()
K.close()
