"""bench_matmat.py — encrypted matrix x matrix product (16-bit, C mod 2^16 as the reference's
default single precision), row blocks sharded over GPUs (cpu-gpu-tfhe_amd/matmat.py).

    python bench_matmat.py --size 8                          # 1 GPU, 8 x 8
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench_matmat.py --size 16

Timed region: every rank's whole circuit evaluation over its row block, bracketed by barrier
+ synchronize, max over ranks; each rank decrypts and checks its block against integer
arithmetic.  One JSON line on rank 0.  Reference (paper Table IX, GTX 1080, BOOTS_matrix-
Multiplication): 4 x 4 5.90 min, 8 x 8 43.95 min, 16 x 16 186.23 min.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))
PAPER_MIN = {4: 5.90, 8: 43.95, 16: 186.23}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8)
    ap.add_argument("--nbits", type=int, default=16)
    ap.add_argument("--double-precision", action="store_true")
    ap.add_argument("--reps", type=int, default=1)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import shard
    import matmat
    import tfhe_amd as T

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    K = T.SecretKeyset()
    ctx = T.Context(K.bk, K.ksk, device=local)
    m = k = n = args.size
    rng = np.random.default_rng(99)                      # same matrices on every rank
    A = rng.integers(0, 2**args.nbits, (m, k))
    Bm = rng.integers(0, 2**args.nbits, (k, n))
    lo, hi = matmat.shard_rows(m, rank, world)
    C, a_w, b_w, c_w = matmat.build(T, k, args.nbits, args.double_precision)
    info = C.info()
    barrier = (lambda: dist.barrier()) if world > 1 else None
    got, t = matmat.run_block_gpu(T, torch, ctx, K, C, a_w, b_w, c_w, A[lo:hi], Bm, args.nbits,
                                  np.random.default_rng(7 + rank), reps=args.reps, barrier=barrier)
    ob = matmat.out_bits(k, args.nbits, args.double_precision)
    want = (A[lo:hi].astype(object) @ Bm.astype(object)) % (2**ob)
    ok = bool(np.array_equal(got, want.astype(np.int64)))
    t_max = shard.max_over_ranks(t, device="cuda")
    if world > 1:
        f = torch.tensor([1.0 if ok else 0.0], device="cuda")
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item() == 1.0)
    if rank == 0:
        line = {"metric": f"encrypted {m}x{k} x {k}x{n} matrix product ({args.nbits}-bit, "
                          f"{'double' if args.double_precision else 'single'} precision) wall time",
                "value": t_max, "unit": "s", "n_gpus": world, "higher_is_better": False, "scaling": "strong",
                "rows_per_rank": hi - lo, "bootstraps_per_element": info["bootstraps"], "depth": info["depth"],
                "bootstraps_per_s_per_gpu": info["bootstraps"] * (hi - lo) * n / t, "correct": ok,
                "paper_gtx1080_s": PAPER_MIN.get(args.size, 0) * 60 or None, "engine": T.version()}
        print(json.dumps(line), flush=True)
    ctx.close()
    K.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
