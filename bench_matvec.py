"""bench_matvec.py — BASELINE config 5: encrypted 64x64 matrix-vector product (16-bit),
rows sharded over GPUs (cpu-gpu-tfhe_amd/matvec.py).  One process per GPU:

    python bench_matvec.py                                   # 1 GPU, all 64 rows
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench_matvec.py
    python bench_matvec.py --rank-of 0 --world-of 8          # rehearse one rank's 1/8 shard
    python bench_matvec.py --multi 0,1,2,3,4,5,6,7           # ONE process, rows sharded over
                                                             # device slots inside the library

Timed region: every rank's whole circuit (all levels), bracketed by barrier + synchronize,
max over ranks.  Each rank decrypts its rows and checks them against integer arithmetic
(no collective on the data path).  Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--cols", type=int, default=64)
    ap.add_argument("--nbits", type=int, default=16)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--rank-of", type=int, default=0, help="single-process rehearsal: act as this rank")
    ap.add_argument("--world-of", type=int, default=1, help="single-process rehearsal: of this many ranks")
    ap.add_argument("--multi", default="", help="one process: device slots of a MultiContext, e.g. 0,1 or "
                    "'all' (tfhe_amd_multi_circuit_run_host shards the rows over them)")
    args = ap.parse_args()
    if args.multi:
        return main_multi(args)
    import torch
    import torch.distributed as dist
    import shard
    import matvec
    import tfhe_amd as T

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    eff_rank, eff_world = (rank, world) if world > 1 else (args.rank_of, args.world_of)

    K = T.SecretKeyset()
    ctx = T.Context(K.bk, K.ksk, device=local)
    data_rng = np.random.default_rng(2024)                 # same matrix / vector on every rank
    A = data_rng.integers(0, 2**args.nbits, (args.rows, args.cols))
    x = data_rng.integers(0, 2**args.nbits, args.cols)
    lo, hi = matvec.shard_rows(args.rows, eff_rank, eff_world)
    C, a_w, x_w, y_w = matvec.build(T, args.cols, args.nbits)
    info = C.info()
    barrier = (lambda: dist.barrier()) if world > 1 else None
    y, t = matvec.run_rows_gpu(T, torch, ctx, K, C, a_w, x_w, y_w, A[lo:hi], x, args.nbits,
                               np.random.default_rng(100 + eff_rank), reps=args.reps, barrier=barrier)
    ok = bool(np.array_equal(y, A[lo:hi] @ x))
    t_max = shard.max_over_ranks(t, device="cuda")
    ok_all = ok
    if world > 1:
        f = torch.tensor([1.0 if ok else 0.0], device="cuda")
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok_all = bool(f.item() == 1.0)
    if rank == 0:
        line = {"metric": f"encrypted {args.rows}x{args.cols} matrix-vector product ({args.nbits}-bit) wall time",
                "value": t_max, "unit": "s", "n_gpus": world, "higher_is_better": False,
                "scaling": "strong", "rows_per_rank": hi - lo,
                "rehearsal": None if world > 1 else {"rank": eff_rank, "world": eff_world},
                "bootstraps_per_row": info["bootstraps"], "depth": info["depth"],
                "bootstraps_per_s_per_gpu": info["bootstraps"] * (hi - lo) / t, "correct": ok_all,
                "engine": T.version(), "reps": args.reps}
        print(json.dumps(line), flush=True)
    ctx.close()
    K.close()
    if world > 1:
        dist.destroy_process_group()


def main_multi(args):
    """All rows from one host process through tfhe_amd_multi_circuit_run_host (matvec.run_rows_multi):
    the library shards the rows over the device slots (one worker thread + key replica each).
    Timed: the whole call (staging in, every level on every device, outputs back)."""
    import torch
    import matvec
    import tfhe_amd as T
    slots = (list(range(torch.cuda.device_count())) if args.multi == "all"
             else [int(d) for d in args.multi.split(",")])
    K = T.SecretKeyset()
    data_rng = np.random.default_rng(2024)
    A = data_rng.integers(0, 2**args.nbits, (args.rows, args.cols))
    x = data_rng.integers(0, 2**args.nbits, args.cols)
    C, a_w, x_w, y_w = matvec.build(T, args.cols, args.nbits)
    info = C.info()
    m = T.MultiContext(K.bk, K.ksk, slots)
    times, ok = [], True
    for r in range(args.reps + 1):                       # the first run warms up (tables, scratch)
        y, t, _, _ = matvec.run_rows_multi(T, m, K, C, a_w, x_w, y_w, A, x, args.nbits, np.random.default_rng(100 + r))
        ok = ok and bool(np.array_equal(y, A @ x))
        if r:
            times.append(t)
    m.close()
    t = float(np.median(times))
    print(json.dumps({"metric": f"encrypted {args.rows}x{args.cols} matrix-vector product ({args.nbits}-bit) wall time",
                      "value": t, "unit": "s", "higher_is_better": False, "mode": "one process, multi-device",
                      "slots": slots, "n_devices": len(set(slots)), "bootstraps_per_row": info["bootstraps"],
                      "depth": info["depth"], "bootstraps_per_s": info["bootstraps"] * args.rows / t,
                      "correct": ok, "engine": T.version(), "reps": args.reps}), flush=True)
    K.close()


if __name__ == "__main__":
    main()
