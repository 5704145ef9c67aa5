"""bench.py — gate bootstraps/s (bootsNAND, N=1024) on MI355X, BASELINE.json's metric.

One "step" = one pass of the hot path over one batch: B independent bootsNAND gates
(gate prologue + 500-step blind rotation + sample extraction + key switch), inputs already
resident in HBM.  Workload = BASELINE.json configs[1]: batch 1024 per GPU (weak scaling: each
rank processes its own shard of independent ciphertexts; no collective on the data path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints ONE JSON line.  Extra objects:
  roofline     : SURVEY.md §8(d)'s figure for the dominant kernel (the blind rotation): its
                 algorithmic key-stream bytes (32 768 000 B of TGSW key per bootstrap, NTT or
                 FFT domain alike) x B / its average time per batch (HIP events the engine
                 records around every launch, on the stream it launches on, live over the K
                 timed steps; one launch per 1024 ciphertexts) vs the 8 TB/s HBM peak;
                 `traffic` = the HBM bytes per launch from the profiles/ PMC data.  Every ciphertext of the batch streams the same key slice
                 per step, so the reads are L2/MALL hits and `frac` can exceed 1; the kernel is
                 in fact bound by fp64 VALU issue, which `roofline.compute` reports: its
                 algorithmic fp64 FLOPs (198 656 per CMux step, FMA = 2) / launch time vs the
                 78.6 TFLOP/s fp64 vector peak.
  cpu_baseline : the CPU restatement (oracle/, same algorithm, exact NTT, OpenMP) timed on
                 this host's cores on a bounded sample of the same workload (rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))

BK_BYTES_PER_BOOTSTRAP = 500 * 4 * 2 * 1024 * 8        # NTT-domain TGSW key stream, 32 768 000 B
KS_BYTES_PER_KEYSWITCH = 1024 * 8 * 501 * 4            # KSK rows, 16 416 768 B
HBM_PEAK_GBPS = 8000.0
# v6 fp64 work per CMux step (blind_rotate_v6.hip), FMA = 2: 4 forward
# transforms x 2304 butterflies x 12 + 2 inverse (640 trivial butterflies x 4 + 1664 x 12 +
# 512-point post-twist x 6) + MAC 2 x 4 x 512 x 7 + partial sums 2048 + mod-2^32 rounding 2048 x 3
INV_FLOPS = 640 * 4 + 1664 * 12 + 512 * 6
FLOPS_PER_CMUX = 4 * 2304 * 12 + 2 * INV_FLOPS + 2 * 4 * 512 * 7 + 2048 + 2048 * 3   # 198 656
FLOPS_PER_BOOTSTRAP = 500 * FLOPS_PER_CMUX
FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 vector (FMA = 2 FLOP), AMD spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="gates per GPU per step")
    ap.add_argument("--gate", default="NAND")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    return ap.parse_args()


def cpu_baseline(bk, ksk, rng, target_s):
    """Oracle (CPU port of the reference path, exact NTT) on all available host threads."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O
    okey = O.OracleKey(bk, ksk, use_ntt=True)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or O.max_threads()
    n = 500

    def run(B):
        a = rng.integers(-2**31, 2**31, (B, n), dtype=np.int64).astype(np.int32)
        b = rng.integers(-2**31, 2**31, B, dtype=np.int64).astype(np.int32)
        t0 = time.perf_counter()
        okey.gate_batch("NAND", a, b, a[::-1].copy(), b[::-1].copy(), nthreads=threads)
        return time.perf_counter() - t0

    t1 = run(threads)                      # warm-up + rate estimate: one gate per thread
    B = max(threads, int(target_s / max(t1, 1e-3)) * threads)
    t = run(B)
    return {"value": B / t, "unit": "gate bootstraps/s", "cores": threads, "kind": "port",
            "sample": f"{B} bootsNAND (random LWE inputs) on {threads} OpenMP threads, {t:.1f} s"}


def pmc_traffic(engine, batch):
    """HBM bytes per blind-rotation launch from the committed rocprofv3 PMC summary
    (profiles/pmc_summary.json, written by scripts/pmc_summary.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per the gfx950 correction for
    16-B-per-lane streaming reads).  None when no summary matches this engine/batch."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        s = json.load(open(path))
    except (OSError, ValueError):
        return None
    k = s.get("kernels", {}).get("blind_rotate")
    if not k or s.get("engine") != engine or s.get("batch") != batch:
        return None
    return k["hbm_bytes_per_launch"]


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import shard
    import tfhe_amd as T

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and int(os.environ.get("RANK", "0")) == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") on the 8-GPU node.  TFHE_AMD_DIST_BACKEND=gloo rehearses the N>1 path with
    # several ranks sharing the GPUs that exist (ranks map to device LOCAL_RANK mod count).
    backend = os.environ.get("TFHE_AMD_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    K = T.SecretKeyset()                   # real keys (seed 314,1592,657), ~1 s on the host
    rng = np.random.default_rng(1000 + rank)
    B = args.batch
    x = rng.integers(0, 2, B)
    y = rng.integers(0, 2, B)
    a_a, a_b = K.encrypt(x, rng)
    b_a, b_b = K.encrypt(y, rng)
    dev = [torch.from_numpy(v).cuda() for v in (a_a, a_b, b_a, b_b)]
    r_a = torch.empty((B, 500), dtype=torch.int32, device="cuda")
    r_b = torch.empty(B, dtype=torch.int32, device="cuda")
    ctx = T.Context(K.bk, K.ksk, device=local)
    ctx.reserve(B)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        ctx.gate_dev(args.gate, r_a, r_b, *dev, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel timing for the roofline: HIP events around each engine launch, recorded by the
    # engine on the stream it launches on, live over the timed steps
    ctx.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, device=red_dev)
    prof = ctx.profile_read()
    ctx.profile_enable(False)

    # correctness guard on the last step's output (truth table; cheap)
    dec = K.decrypt(r_a.cpu().numpy(), r_b.cpu().numpy())
    truth_ok = bool(np.array_equal(dec, 1 - (x & y))) if args.gate == "NAND" else None

    br_ms = prof["br_ms"] / max(1, prof["br_launches"])
    ks_ms = prof["ks_ms"] / max(1, prof["ks_launches"])
    key_gbps = B * BK_BYTES_PER_BOOTSTRAP / (br_ms * 1e-3) / 1e9
    fft = "fft64" in T.version()
    roof = {"bound": "hbm", "achieved": key_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": key_gbps / HBM_PEAK_GBPS, "traffic": pmc_traffic(T.version(), B),
            "kernel": "k_blind_rotate_v" + T.version().split("br-v")[1].split(" ")[0], "kernel_ms": br_ms,
            "keyswitch_ms": ks_ms, "algorithmic_bytes_per_launch": B * BK_BYTES_PER_BOOTSTRAP,
            "note": "achieved counts every ciphertext's full key stream; the batch shares each key "
                    "slice through L2 (hit rate 99 %), so frac > 1 is possible and traffic (real HBM "
                    "bytes) is ~1 % of it; the kernel is SIMD-bound, see compute (DESIGN.md 5.1)"}
    if fft:
        tflops = B * FLOPS_PER_BOOTSTRAP / (br_ms * 1e-3) / 1e12
        roof["compute"] = {"bound": "valu-fp64", "achieved": tflops, "peak": FP64_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": tflops / FP64_PEAK_TFLOPS,
                           "flops_per_launch": B * FLOPS_PER_BOOTSTRAP}

    value = shard.weak_scaling_value(B, world, args.steps, elapsed)
    line = {
        "metric": "gate bootstraps/sec (bootsNAND, N=1024)",
        "value": value,
        "unit": "gate bootstraps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("f64 (FFT external product; Torus32 in/out, rounded products exact)" if fft
                  else "int32 (Torus32; exact 2x27-bit CRT NTT)"),
        "data": "synthetic: random bits encrypted under keys generated from seed {314,1592,657}",
        "config": {"workload": f"batch of {B} independent boots{args.gate} per GPU (BASELINE configs[1])",
                   "batch_per_gpu": B, "gate": args.gate, "params": "n=500 N=1024 k=1 l=2 Bgbit=10 ks_t=8 ks_basebit=2",
                   "parallelism": f"shard{world} (independent ciphertexts, no collective)"},
        "roofline": roof,
        "truth_table_ok": truth_ok,
        "engine": T.version(),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(K.bk, K.ksk, np.random.default_rng(5), args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    K.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
