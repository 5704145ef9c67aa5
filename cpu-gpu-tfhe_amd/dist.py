"""One process per GPU over torch.distributed: a batch of independent gates
held by rank 0 is scattered in contiguous shards (shard.shard_range), every rank evaluates its
shard on its own device context (keys replicated), and rank 0 gathers the results.

The exchange is host-side ciphertext I/O (2 004 B per sample), not a collective of the compute
path: with the gloo backend it moves CPU tensors; with RCCL ("nccl") the shards travel as device
tensors over xGMI.  Shards are padded to the largest one because torch.distributed's scatter and
gather move equal-sized tensors; the padding rows are never evaluated.  The single-process
alternative for C/C++ callers is the library's multi-device context (tfhe_amd_multi_*,
tfhe_gpu_boots_batch) — the same shard arithmetic, one worker thread per device.
"""
import numpy as np

import shard

N_LWE = 500


def run_sharded(evaluate, inputs, rank, world, device=None):
    """inputs: on rank 0 a tuple of SoA arrays (a [B][500], b [B], ... pairs, all with the same B),
    elsewhere None.  evaluate(*shard_arrays) -> (res_a [n][500], res_b [n]) on each rank's shard.
    Returns the gathered (res_a, res_b) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    meta = torch.zeros(2, dtype=torch.int64, device=device)
    if rank == 0:
        meta[0] = inputs[0].shape[0]
        meta[1] = len(inputs)
    dist.broadcast(meta, 0)
    B, nin = int(meta[0]), int(meta[1])
    spans = [shard.shard_range(B, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in spans) if B else 0
    lo, hi = spans[rank]
    mine = []
    for k in range(nin):
        width = N_LWE if k % 2 == 0 else 1
        buf = torch.zeros((cap, width), dtype=torch.int32, device=device)
        chunks = None
        if rank == 0:
            arr = np.asarray(inputs[k], dtype=np.int32).reshape(B, width)
            chunks = []
            for a, b in spans:
                c = torch.zeros((cap, width), dtype=torch.int32, device=device)
                c[: b - a] = torch.from_numpy(arr[a:b])
                chunks.append(c)
        dist.scatter(buf, chunks, src=0)
        part = buf[: hi - lo].cpu().numpy()
        mine.append(part if width > 1 else part.reshape(-1))
    res_a, res_b = evaluate(*mine) if hi > lo else (np.zeros((0, N_LWE), np.int32), np.zeros(0, np.int32))
    out = []
    for res, width in ((res_a, N_LWE), (res_b, 1)):
        buf = torch.zeros((cap, width), dtype=torch.int32, device=device)
        buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(res, dtype=np.int32).reshape(hi - lo, width))
        got = [torch.zeros((cap, width), dtype=torch.int32, device=device) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, got, dst=0)
        if rank == 0:
            full = np.concatenate([g[: b - a].cpu().numpy() for g, (a, b) in zip(got, spans)])
            out.append(full if width > 1 else full.reshape(-1))
    return tuple(out) if rank == 0 else None
