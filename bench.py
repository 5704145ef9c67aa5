"""bench.py — gate bootstraps/s (bootsNAND, N=1024) on MI355X, BASELINE.json's metric.

One "step" = one pass of the hot path over one batch: B independent bootsNAND gates
(gate prologue + 500-step blind rotation + sample extraction + key switch), inputs already
resident in HBM.  Workload = BASELINE.json configs[1]: batch 1024 per GPU (weak scaling: each
rank processes its own shard of independent ciphertexts; no collective on the data path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints ONE JSON line.  Extra objects:
  roofline     : the dominant kernel (the blind rotation) against the roofline that binds it,
                 fp64 VALU issue: its algorithmic fp64 FLOPs (198 656 per CMux step, FMA = 2,
                 x 500 steps x B) / its average launch time (HIP events the engine records
                 around every launch, on the stream it launches on, live over the K timed steps)
                 vs the 78.6 TFLOP/s fp64 vector peak.  `traffic` = HBM bytes per launch from
                 the committed rocprofv3 PMC passes (profiles/pmc_summary.json).
                 `hbm` is SURVEY.md §8(d)'s key-stream view of the same launch: the measured
                 HBM bytes (PMC) / launch time vs 8 TB/s, next to the streaming model's
                 algorithmic bytes (every ciphertext streaming the 32.768 MB key; the batch
                 shares each key slice through L2, so those are cache hits, not HBM reads).
                 `clock` = the shader clock sampled during a sustained run (amd-smi), and the
                 fp64 fraction at that clock.  `sustained` = the fp64 FMA rate the chip holds
                 under its power limit (tfhe_amd_fp64_ceiling: pure register FMA chains, at the
                 kernel's 2 waves per SIMD and at 8) and the kernel's fraction of each.
  batches      : the same step at B = 1, 128, 256, 512 and 4096 per GPU (BASELINE metric's other
                 batch sizes; 128 / 512 = the per-GPU shapes of the strong-scaled 1024 / 4096 at N = 8)
  strong       : global batches 1024 and 4096, each split over the ranks (BASELINE: 1..8 GPUs)
  host_path    : (1 rank) the host-pointer API at B = 1024 and 4096: inputs and results in host
                 memory, PCIe-inclusive, median call — for comparison, never `value`; `host_path`
                 = pageable arrays staged by the library, `host_path_pinned` = caller-owned
                 page-locked arrays (tfhe_amd_host_alloc)
  circuits     : BASELINE configs 3-5 wall time through the circuit engine (32-bit add, 16 x 16
                 multiply x 256, 64 x 64 16-bit matrix-vector with rows sharded over the ranks)
  cpu_baseline : the optimized CPU port (oracle/cpu_fft.c: fp64 FFT external product, the
                 spqlios algorithm class, AVX2/AVX-512, OpenMP over gates; Torus32-identical to
                 the exact oracle) timed on this host's cores on a bounded sample (rank 0, N=1),
                 with its single-core ms per bootstrap and the host CPU model.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))

BK_BYTES_PER_BOOTSTRAP = 500 * 4 * 2 * 1024 * 8        # FFT/NTT-domain TGSW key stream, 32 768 000 B
KS_BYTES_PER_KEYSWITCH = 1024 * 8 * 501 * 4            # KSK rows, 16 416 768 B
IO_BYTES_PER_GATE = 2 * 2004 + 4100                    # two LWE inputs read + one extracted sample written
HBM_PEAK_GBPS = 8000.0
# v6 fp64 work per CMux step (blind_rotate_v6.hip), FMA = 2: 4 forward
# transforms x 2304 butterflies x 12 + 2 inverse (640 trivial butterflies x 4 + 1664 x 12 +
# 512-point post-twist x 6) + MAC 2 x 4 x 512 x 7 + partial sums 2048 + mod-2^32 rounding 2048 x 3
INV_FLOPS = 640 * 4 + 1664 * 12 + 512 * 6
FLOPS_PER_CMUX = 4 * 2304 * 12 + 2 * INV_FLOPS + 2 * 4 * 512 * 7 + 2048 + 2048 * 3   # 198 656
FLOPS_PER_BOOTSTRAP = 500 * FLOPS_PER_CMUX
# the textbook count: 10 FLOP per non-trivial radix-2 butterfly (one complex multiply = 6, two
# complex adds = 4) instead of the 6 FMAs = 12 the kernel issues; `roofline.frac_10flop`
FLOPS_PER_CMUX_10 = 4 * 2304 * 10 + 2 * (640 * 4 + 1664 * 10 + 512 * 6) + 2 * 4 * 512 * 7 + 2048 + 2048 * 3  # 173 568
FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 vector (FMA = 2 FLOP) at the 2.4 GHz peak clock
PEAK_CLOCK_MHZ = 2400.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first: the clock and power state settle within ~10 (2: -2 %%)")
    ap.add_argument("--batch", type=int, default=1024, help="gates per GPU per step")
    ap.add_argument("--gate", default="NAND")
    ap.add_argument("--extra-batches", default="1,128,256,512,4096",
                    help="per-GPU batch sizes also timed ('none' = none); 128 / 512 = the per-GPU shapes of the "
                         "global 1024 / 4096 at N = 8")
    ap.add_argument("--strong-batch", default="1024,4096",
                    help="global batches each split over the ranks ('0' or 'none' = skip)")
    ap.add_argument("--no-circuits", action="store_true", help="skip the configs 3-5 circuit leg")
    ap.add_argument("--host-batches", default="1024,4096",
                    help="PCIe-inclusive host-pointer path also timed at these batches (rank 0 of a 1-rank run; 'none')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clock", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the sustained fp64 ceiling measurement")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-multi", action="store_true",
                    help="skip the one-process multi-device leg (only runs when several GPUs are visible)")
    ap.add_argument("--multi-devices", default="",
                    help="device slots of the one-process multi-device leg (default: every visible GPU; "
                         "e.g. 0,0 rehearses two slots on one GPU)")
    ap.add_argument("--multi-only", action="store_true", help=argparse.SUPPRESS)   # the child of run_multi_child
    ap.add_argument("--parity-samples", type=int, default=128,
                    help="outputs of the timed batch compared Torus32-for-Torus32 with the exact oracle")
    return ap.parse_args()


# ------------------------------------------------------------------------------- CPU side

def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity}


def cpu_threads():
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share():
    """What caps the CPU baseline's thread count on this host: OMP_NUM_THREADS (the GPU pool sets
    it to each GPU's share of the host, 16), the cgroup CPU quota, the affinity mask; plus the
    physical core count (unique (socket, core) pairs) for the full-socket extrapolation."""
    out = {"omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        out["cgroup_cpu_quota"] = None if q[0] == "max" else float(q[0]) / float(q[1])
    except (OSError, ValueError, IndexError):
        out["cgroup_cpu_quota"] = None
    cores, phys = set(), None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":")[1].strip()))
    except OSError:
        pass
    out["physical_cores"] = len(cores) or None
    return out


def cpu_baseline(bk, ksk, inputs, gpu_out, target_s):
    """The optimized CPU port (oracle/cpu_fft.c) on the SAME inputs as the timed GPU batch (the
    batch repeated to fill ~target_s), on the threads this process may use (OMP_NUM_THREADS, else
    its CPU affinity), plus a single-thread sample.  Its outputs are also compared word for word
    with the GPU's outputs of that batch (the port is Torus32-identical to the exact oracle,
    tests/test_cpu_baseline.py)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O
    fk = O.CpuFftKey(bk, ksk)
    threads = cpu_threads()
    a_a, a_b, b_a, b_b = inputs
    B = a_a.shape[0]
    g_a, g_b = gpu_out

    def run(lo, hi, th):
        t0 = time.perf_counter()
        r = fk.gate_batch("NAND", a_a[lo:hi], a_b[lo:hi], b_a[lo:hi], b_b[lo:hi], nthreads=th)
        return time.perf_counter() - t0, r

    run(0, min(B, threads), threads)                  # warm-up (thread team, key pages)
    t1, (c_a, c_b) = run(0, B, threads)               # the whole timed batch once
    mismatches = int(np.sum(np.any(c_a != g_a, axis=1) | (c_b != g_b)))
    reps = max(0, int(target_s / max(t1, 1e-3)) - 1)
    t, n = t1, B
    for _ in range(reps):                             # the same batch again, to fill the sample
        dt, _ = run(0, B, threads)
        t += dt
        n += B
    # single-core figure: 32 bootstraps per sample, median of 5 samples (a 2 x 4 sample varied
    # 7.8-10.5 ms box to box in round 3); the spread of the 5 is reported beside it
    run(0, 1, 1)
    n1 = min(B, 32)
    singles = sorted(run(0, n1, 1)[0] / n1 for _ in range(5))
    single = singles[2]
    share = cpu_share()
    out = {"value": n / t, "unit": "gate bootstraps/s", "cores": threads, "kind": "port",
           "sample": f"the timed GPU batch's {B} bootsNAND inputs, {n // B} pass(es) = {n} bootstraps on "
                     f"{threads} OpenMP threads, {t:.1f} s",
           "engine": "optimized fp64-FFT port of the reference CPU path (oracle/cpu_fft.c; spqlios "
                     "algorithm class, AVX2/AVX-512, OpenMP over gates; Torus32-identical to the exact oracle)",
           "same_inputs_as_gpu": True, "outputs_vs_gpu": {"checked": B, "mismatches": mismatches},
           "single_core_ms_per_bootstrap": single * 1e3,
           "single_core_sample": {"bootstraps": n1, "samples": 5, "statistic": "median",
                                  "min_ms": singles[0] * 1e3, "max_ms": singles[-1] * 1e3},
           "per_thread_ms_per_bootstrap": threads * t / n * 1e3,
           "paper_single_core_ms_per_gate": 43.8,
           "max_round_error": fk.max_round_error(),
           "thread_cap": share,
           "thread_cap_note": "threads = OMP_NUM_THREADS, which the GPU pool sets to each GPU's share of "
                              "the host's CPUs (16 per GPU); nproc / affinity show the whole machine"}
    if share.get("physical_cores"):
        out["full_socket_extrapolation"] = {
            "value": share["physical_cores"] * 1e3 / (single * 1e3), "cores": share["physical_cores"],
            "note": "single-core rate x physical cores (linear; an upper bound, not measured)"}
    out.update(host_info())
    return out


# ------------------------------------------------------------------------------- GPU side

def pmc_traffic(engine, batch):
    """HBM bytes per blind-rotation launch from the committed rocprofv3 PMC summary
    (profiles/pmc_summary.json, written by scripts/pmc_summary.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per the gfx950 correction for
    16-B-per-lane streaming reads).  None when no summary matches this engine/batch."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        s = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    k = s.get("kernels", {}).get("blind_rotate")
    if not k or s.get("engine") != engine or s.get("batch") != batch:
        return None, None
    return k["hbm_bytes_per_launch"], s.get("source")


def _gfx_clock_mhz(obj):
    """Current GFX clock(s) from `amd-smi metric --clock --json` (tolerant walk)."""
    vals = []

    def walk(o, path):
        if isinstance(o, dict):
            for k, v in o.items():
                walk(v, path + [str(k).lower()])
        elif isinstance(o, list):
            for v in o:
                walk(v, path)
        else:
            p = "/".join(path)
            if "gfx" in p and ("clk" in p or "clock" in p) and "min" not in p and "max" not in p \
                    and "lock" not in p.replace("clock", "") and ("cur" in p or p.endswith("clk/value")):
                try:
                    vals.append(float(o))
                except (TypeError, ValueError):
                    pass
    walk(obj, [])
    return vals


def sample_clock(device, run_step, seconds=2.0):
    """Shader clock under the bench's own sustained load: steps run back to back on the GPU
    while another thread samples amd-smi.  Returns {"mhz": median, "samples": n} or None."""
    samples = []
    stop = threading.Event()

    def poll():
        while not stop.is_set():
            try:
                r = subprocess.run(["amd-smi", "metric", "-g", str(device), "--clock", "--json"],
                                   capture_output=True, text=True, timeout=10)
                v = _gfx_clock_mhz(json.loads(r.stdout)) if r.returncode == 0 and r.stdout.strip() else []
                v = [x for x in v if 100.0 < x < 5000.0]
                if v:
                    samples.append(sum(v) / len(v))
            except Exception:   # no amd-smi / unparsable output: no clock figure
                return
    th = threading.Thread(target=poll, daemon=True)
    t_end = time.perf_counter() + seconds
    run_step()
    th.start()
    while time.perf_counter() < t_end:
        run_step()
    stop.set()
    th.join(timeout=15)
    if not samples:
        return None
    samples.sort()
    return {"mhz": samples[len(samples) // 2], "samples": len(samples)}


def multi_device_leg(T, torch, K, args, rng):
    """B = args.batch gates per device on every visible device from this one process: a
    MultiContext over all devices, each shard resident in its device's HBM, K steps of
    multi.gate_dev + multi.sync timed; the NAND truth table of every shard checked after."""
    devs = ([int(d) for d in args.multi_devices.split(",")] if args.multi_devices
            else list(range(torch.cuda.device_count())))
    n = len(devs)
    m = T.MultiContext(K.bk, K.ksk, devs)
    B = args.batch
    shards, bits = [], []
    for d in devs:
        x, y = rng.integers(0, 2, B), rng.integers(0, 2, B)
        a_a, a_b = K.encrypt(x, rng)
        b_a, b_b = K.encrypt(y, rng)
        dev = [torch.from_numpy(v).to(f"cuda:{d}") for v in (a_a, a_b, b_a, b_b)]
        r_a = torch.empty((B, 500), dtype=torch.int32, device=f"cuda:{d}")
        r_b = torch.empty(B, dtype=torch.int32, device=f"cuda:{d}")
        shards.append([r_a, r_b] + dev)
        bits.append((x, y))
    for _ in range(max(1, args.warmup)):
        m.gate_dev(args.gate, shards)
    m.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.gate_dev(args.gate, shards)
    m.sync()
    el = time.perf_counter() - t0
    ok = None
    if args.gate == "NAND":
        ok = all(np.array_equal(K.decrypt(sh[0].cpu().numpy(), sh[1].cpu().numpy()), 1 - (x & y))
                 for sh, (x, y) in zip(shards, bits))
    m.close()
    return {"devices": n, "batch_per_device": B, "steps": args.steps, "ms_per_step": el / args.steps * 1e3,
            "value": n * B * args.steps / el, "truth_table_ok": ok,
            "api": "tfhe_amd_multi_gate_batch_dev + tfhe_amd_multi_sync (one process, one key replica per device)"}


def run_multi_child(args):
    """The multi-device leg in a child process under a 150 s limit, so that a fault or hang on a
    many-GPU host costs that leg, never the headline line (the parent has synchronized its own
    GPU work and waits idle)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--multi-only", "--batch", str(args.batch), "--steps",
           str(args.steps), "--warmup", str(args.warmup), "--gate", args.gate]
    if args.multi_devices:
        cmd += ["--multi-devices", args.multi_devices]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 150 s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"child exit {r.returncode}: {r.stderr[-400:]}"}
    return json.loads(lines[-1])


def multi_only(args):
    import torch
    import tfhe_amd as T
    K = T.SecretKeyset()
    try:
        out = multi_device_leg(T, torch, K, args, np.random.default_rng(7000))
    except Exception as e:
        out = {"error": repr(e)[:500]}
    print(json.dumps(out), flush=True)
    K.close()


def circuits_leg(T, torch, ctx, K, rank, world, dist, red_dev, rows5=64, shard5=8):
    """BASELINE configs 3-5 through the batched circuit engine (csrc/circuit.cpp; SURVEY.md §8(d):
    "plus wall time for configs 3-5").  Every level of a circuit is one blind-rotation launch over
    (gates x instances) plus one key switch; inputs are encrypted and resident in HBM, the timed
    region is the whole circuit between synchronize (+ barrier) calls, max over ranks; outputs are
    decrypted afterwards and checked against integer arithmetic on every rank.
      config 3: 32-bit ripple-carry add, one instance per rank (Cipher.cpp:348-392's operator+;
                a dependency chain: replicas only at N > 1)
      config 4: 16 x 16 multiply, 256 instances per rank (main.cu:1483-1579's multiplyLweSamples)
      config 5: 64 x 64 16-bit matrix-vector product, rows sharded contiguously over the ranks
                (main.cu:2342-2462, matrixUtility.cu:65-96); at N = 1 also one 8-row shard alone,
                the per-rank work of the 8-GPU run."""
    import matvec
    import shard
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    rng = np.random.default_rng(5000 + rank)
    stream = torch.cuda.current_stream().cuda_stream

    def all_ok(ok):
        return bool(shard.max_over_ranks(0.0 if ok else 1.0, device=red_dev) == 0.0)

    def timed_runs(C, B, wa, wb, reps, warm=True):
        if warm:   # compiles the schedule, uploads its tables, sizes the scratch
            C.run_dev(ctx, B, wa, wb, stream)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            C.run_dev(ctx, B, wa, wb, stream)
            torch.cuda.synchronize()
            barrier()
            ts.append(time.perf_counter() - t0)
        return shard.max_over_ranks(float(np.median(ts)), device=red_dev)

    def upload(C, wires_bits, B):
        n_w = C.info()["wires"]
        wa = torch.zeros((n_w, B, 500), dtype=torch.int32, device="cuda")
        wb = torch.zeros((n_w, B), dtype=torch.int32, device="cuda")
        for w, plane in wires_bits.items():
            ea, eb = K.encrypt(plane, rng)
            wa[w] = torch.from_numpy(ea).cuda()
            wb[w] = torch.from_numpy(eb).cuda()
        return wa, wb

    def binop(name, build, nbits, B, reps, ref, what):
        C = T.Circuit()
        a, b = C.inputs(nbits), C.inputs(nbits)
        outs = build(C, a, b)
        info = C.info()
        x, y = rng.integers(0, 2**nbits, B), rng.integers(0, 2**nbits, B)
        bits = dict(zip(a, T.bits_of(x, nbits)))
        bits.update(zip(b, T.bits_of(y, nbits)))
        wa, wb = upload(C, bits, B)
        t = timed_runs(C, B, wa, wb, reps)
        ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
        ok = all_ok(np.array_equal(T.int_of([K.decrypt(ha[w], hb[w]) for w in outs]), ref(x, y)))
        C.close()
        return {"what": what, "instances_per_rank": B, "seconds": t, "bootstraps_per_instance": info["bootstraps"],
                "depth": info["depth"], "bootstraps_per_s": info["bootstraps"] * B * world / t,
                "statistic": f"median of {reps} runs, max over ranks", "correct": ok}

    out = {}
    out["config3_add32"] = binop("add32", lambda C, a, b: (lambda s: s[0] + [s[1]])(C.add(a, b)), 32, 1, 5,
                                 lambda x, y: x + y, "32-bit ripple-carry add, one instance per rank")
    out["config3_add32_prefix"] = binop("add32p", lambda C, a, b: (lambda s: s[0] + [s[1]])(C.add_prefix(a, b)), 32, 1,
                                        5, lambda x, y: x + y,
                                        "the same 32-bit addition as a parallel-prefix circuit (fewer levels, "
                                        "more gates per level): what a caller gains by not following the ripple")
    out["config4_mul16_b256"] = binop("mul16", lambda C, a, b: C.mul(a, b), 16, 256, 2, lambda x, y: x * y,
                                      "16 x 16 -> 32-bit multiply (Dadda tree), 256 instances per rank")
    # config 5: the same matrix and vector on every rank, this rank's rows
    data = np.random.default_rng(2024)
    A = data.integers(0, 2**16, (rows5, 64))
    xv = data.integers(0, 2**16, 64)
    C, a_w, x_w, y_w = matvec.build(T, 64, 16)
    info = C.info()

    def rows_run(lo, hi, warm):
        B = hi - lo
        wa, wb = upload(C, matvec.instance_inputs(T, a_w, x_w, A[lo:hi], xv, 16), B)
        t = timed_runs(C, B, wa, wb, 1, warm=warm)
        ha, hb = wa.cpu().numpy(), wb.cpu().numpy()
        ok = np.array_equal(T.int_of([K.decrypt(ha[w], hb[w]) for w in y_w]), A[lo:hi] @ xv)
        return t, ok

    c5 = {"matrix": f"{rows5} x 64, 16-bit entries, 64-entry vector; {len(y_w)}-bit outputs",
          "bootstraps_per_row": info["bootstraps"], "depth": info["depth"]}
    if world == 1:
        # one 8-row shard first (warms the schedule's tables), then all rows, the 64-row call
        # growing the extracted-sample scratch once (one hipMalloc)
        ts, ok_s = rows_run(0, shard5, True)
        t, ok = rows_run(0, rows5, False)
        c5.update({"rows_per_rank": rows5, "seconds": t, "bootstraps_per_s": info["bootstraps"] * rows5 / t,
                   "correct": bool(ok and ok_s),
                   "shard_of_8": {"rows": shard5, "seconds": ts, "bootstraps_per_s": info["bootstraps"] * shard5 / ts,
                                  "what": "one rank's share of the 8-GPU run, on this GPU"}})
    else:
        lo, hi = matvec.shard_rows(rows5, rank, world)
        if hi == lo:   # more ranks than rows (world > 64): this rank repeats row 0, so every rank
            lo, hi = 0, 1   # still joins the leg's barriers and reductions
        rows_run(lo, min(hi, lo + 1), True)                 # schedule tables + warm-up, one row
        t, ok = rows_run(lo, hi, False)
        c5.update({"rows_per_rank": hi - lo, "seconds": t, "bootstraps_per_s": info["bootstraps"] * rows5 / t,
                   "correct": all_ok(ok), "scaling": "strong (rows sharded over the ranks, no collective)"})
    C.close()
    out["config5_matvec64"] = c5
    out["note"] = ("circuit engine: one blind-rotation launch + one key switch per bootstrap level over all "
                   "gates x instances (DESIGN.md §9); seconds exclude encryption / decryption")
    return out


def headline_parity(K, gate, rec, nsamp, rank, world, red_dev):
    """Torus32 parity of the timed batch itself: `nsamp` of its outputs (launch seams, rounds and
    a seeded random sample) against the exact CPU oracle (tests/oracle_ctypes.py, test-only
    checker), max-reduced over the ranks."""
    import shard
    a_a, a_b, b_a, b_b = rec["inputs"]
    g_a, g_b = rec["outputs"]
    B = a_a.shape[0]
    if B == 0 or nsamp <= 0:
        return {"checked_per_rank": 0, "mismatches": 0}
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ctypes as O
    seams = [i for i in (0, 1, 63, 64, 127, 128, 255, 256, 257, 511, 512, 513, 767, 768, 1023, 1024, 1025,
                         2047, 2048, 4095) if i < B] + [B - 1]
    rng = np.random.default_rng(4242 + rank)
    rest = rng.choice(B, min(B, max(0, nsamp - len(seams))), replace=False)
    idx = np.unique(np.concatenate([np.array(seams, dtype=np.int64), rest.astype(np.int64)]))
    ok = O.OracleKey(K.bk, K.ksk, use_ntt=True)
    o_a, o_b = ok.gate_batch(gate, a_a[idx], a_b[idx], b_a[idx], b_b[idx])
    local_bad = int(np.sum(np.any(g_a[idx] != o_a, axis=1) | (g_b[idx] != o_b)))
    bad = int(shard.max_over_ranks(float(local_bad), device=red_dev)) if world > 1 else local_bad
    return {"checked_per_rank": int(len(idx)), "mismatches": bad, "mismatches_local": local_bad,
            "vs": "exact CPU oracle (oracle/tfhe_oracle.c)",
            "what": "outputs of the timed batch, Torus32 words (a[500], b); mismatches = max over ranks"}


def device_identity(torch, local):
    """This rank's GPU as the runtime reports it: PCI domain:bus:device and UUID."""
    p = torch.cuda.get_device_properties(local)
    uuid = getattr(p, "uuid", None)
    return {"device": local, "name": p.name, "cus": p.multi_processor_count,
            "pci": "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                       getattr(p, "pci_device_id", 0)),
            "uuid": None if uuid is None else str(uuid)}


def rank_block(dist, torch, local, backend, rank, world, truth_ok, parity, strong_ok, ms_per_step):
    """Gathered from every rank (all_gather_object: the only collective besides the timing max): its
    device identity, its headline step time, truth table and oracle parity, and its strong-leg truth
    table.  With RCCL ("nccl") every rank must sit on its own physical GPU: asserted on the PCI ids
    and UUIDs (a gloo rehearsal may share one GPU between ranks) — reported, and warned about on
    stderr rather than raised, so that a partitioned part whose logical GPUs share a PCI function
    cannot abort the scaling run (RCCL itself refuses two ranks on one device)."""
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), **device_identity(torch, local),
            "ms_per_step": ms_per_step, "truth_table_ok": truth_ok,
            "parity_checked": parity.get("checked_per_rank"), "parity_mismatches_local": parity.get("mismatches_local"),
            "strong_truth_table_ok": strong_ok}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    allr.sort(key=lambda r: r["rank"])
    pcis, uuids = [r["pci"] for r in allr], [r["uuid"] for r in allr]
    distinct = len(set(pcis)) == world or (None not in uuids and len(set(uuids)) == world)
    if backend == "nccl" and not distinct and rank == 0:
        print(f"warning: RCCL world of {world} ranks but devices are not distinct: {pcis} {uuids}", file=sys.stderr)
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "distinct_devices": distinct,
            "per_rank": allr}


def main():
    args = parse()
    if args.multi_only:
        return multi_only(args)
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
    ctx = T.Context(K.bk, K.ksk, device=local)
    stream = torch.cuda.current_stream().cuda_stream

    def make_batch(B):
        x = rng.integers(0, 2, B)
        y = rng.integers(0, 2, B)
        a_a, a_b = K.encrypt(x, rng)
        b_a, b_b = K.encrypt(y, rng)
        dev = [torch.from_numpy(v).cuda() for v in (a_a, a_b, b_a, b_b)]
        r_a = torch.empty((B, 500), dtype=torch.int32, device="cuda")
        r_b = torch.empty(B, dtype=torch.int32, device="cuda")
        ctx.reserve(B)
        return x, y, dev, r_a, r_b, (a_a, a_b, b_a, b_b)

    local_el = [0.0]   # this rank's own elapsed time of the last timed() (before the max over ranks)

    def timed(B, steps, warmup, profile=False, warm_s=0.0):
        """W warmup + K timed steps of batch B, barrier + synchronize on both sides, max over
        ranks; returns (elapsed_s, profile dict, truth_ok, step, batch record).  warm_s: keep
        warming up at this batch for at least that long (a leg that follows another batch size
        starts from the clock and power state the previous load left)."""
        x, y, dev, r_a, r_b, host_in = make_batch(B)

        def step():
            if B > 0:
                ctx.gate_dev(args.gate, r_a, r_b, *dev, stream=stream)
        t_w = time.perf_counter()
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        while B > 0 and time.perf_counter() - t_w < warm_s:
            for _ in range(8):
                step()
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if profile:
            # kernel timing for the roofline: HIP events around each engine launch, recorded by
            # the engine on the stream it launches on, live over the timed steps
            ctx.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        local_el[0] = time.perf_counter() - t0
        el = shard.max_over_ranks(local_el[0], device=red_dev)
        prof = None
        if profile:
            prof = ctx.profile_read()
            ctx.profile_enable(False)
        ok = None
        out = (r_a.cpu().numpy(), r_b.cpu().numpy()) if B > 0 else None
        if args.gate == "NAND" and B > 0:
            dec = K.decrypt(*out)
            ok = bool(np.array_equal(dec, 1 - (x & y)))
        return el, prof, ok, step, {"inputs": host_in, "outputs": out, "kernels": ctx.last_kernels()}

    B = args.batch
    elapsed, prof, truth_ok, main_step, rec = timed(B, args.steps, args.warmup, profile=True)
    local_ms_per_step = local_el[0] / args.steps * 1e3
    parity = headline_parity(K, args.gate, rec, args.parity_samples, rank, world, red_dev)

    br_ms = prof["br_ms"] / max(1, prof["br_launches"])
    ks_ms = prof["ks_ms"] / max(1, prof["ks_launches"])
    fft = "fft64" in T.version()
    kernel = "k_blind_rotate_v" + T.version().split("br-v")[1].split(" ")[0]
    traffic, traffic_src = pmc_traffic(T.version(), B)
    unique = BK_BYTES_PER_BOOTSTRAP + B * IO_BYTES_PER_GATE
    hbm = {"achieved": None if traffic is None else traffic / (br_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBPS,
           "unit": "GB/s", "frac": None if traffic is None else traffic / (br_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
           "traffic_bytes_per_launch": traffic, "traffic_source": traffic_src,
           "unique_bytes_per_launch": unique,
           "refetch_ratio": None if traffic is None else traffic / unique,
           "streaming_model_bytes_per_launch": B * BK_BYTES_PER_BOOTSTRAP,
           "streaming_model_GBps": B * BK_BYTES_PER_BOOTSTRAP / (br_ms * 1e-3) / 1e9,
           "note": "traffic = HBM bytes from PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch; "
                   "refetch_ratio = traffic / (key once + ciphertext I/O): each XCD's L2 refills the "
                   "key; the streaming model counts every ciphertext's key stream, served from L2"}
    if fft:
        tflops = B * FLOPS_PER_BOOTSTRAP / (br_ms * 1e-3) / 1e12
        tflops10 = B * 500 * FLOPS_PER_CMUX_10 / (br_ms * 1e-3) / 1e12
        roof = {"bound": "valu-fp64", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tflops / FP64_PEAK_TFLOPS, "flop_convention": "frac: 12 FLOP per radix-2 butterfly (the 6 "
                "v_fma_f64 the kernel issues, FMA = 2); frac_10flop: the textbook 10",
                "achieved_10flop": tflops10, "frac_10flop": tflops10 / FP64_PEAK_TFLOPS,
                "traffic": traffic, "kernel": kernel, "kernel_ms": br_ms,
                "keyswitch_ms": ks_ms, "flops_per_launch": B * FLOPS_PER_BOOTSTRAP,
                "flops_per_cmux_step": FLOPS_PER_CMUX, "hbm": hbm}
    else:   # exact-NTT generations: integer VALU bound; report the key-stream view only
        roof = {"bound": "valu-int", "achieved": None, "peak": None, "unit": None, "frac": None,
                "traffic": traffic, "kernel": kernel, "kernel_ms": br_ms, "keyswitch_ms": ks_ms, "hbm": hbm}

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
        "parity": parity,
        "kernels": rec["kernels"],
        "engine": T.version(),
    }

    # the metric's other batch sizes (per GPU, weak scaling like the headline)
    extras = {}
    for s in (v for v in args.extra_batches.split(",") if v.strip() and v.strip() not in ("none", "''")):
        b = int(s)
        if b == B or b <= 0:
            continue
        steps = max(3, min(args.steps, int(200 / b) + 5)) if b < 64 else max(3, args.steps // 2)
        # warm-up at the leg's own batch: at least 3 steps and 0.3 s (after the headline's batch the
        # chip's clock needs a moment to settle to this load: B = 512 read 5 % low with 3 steps)
        el, pr, ok, _, _ = timed(b, steps, 3, profile=True, warm_s=0.3)
        extras[str(b)] = {"value": shard.weak_scaling_value(b, world, steps, el), "ms_per_step": el / steps * 1e3,
                          "steps": steps, "kernel_ms": pr["br_ms"] / max(1, pr["br_launches"]),
                          "keyswitch_ms": pr["ks_ms"] / max(1, pr["ks_launches"]), "truth_table_ok": ok}
    if extras:
        line["batches"] = extras
    # strong scaling of each global batch over the ranks (contiguous shards, shard.py): the metric's
    # own 1024 (128 per GPU at N = 8) and 4096 (512 per GPU)
    strong_ok = {}
    strong = {}
    for s_ in args.strong_batch.split(","):
        if not s_.strip() or s_.strip() in ("0", "none", "''"):
            continue
        gb = int(s_)
        lo, hi = shard.shard_range(gb, rank, world)
        steps = max(3, args.steps // 2)
        el, _, ok_, _, _ = timed(hi - lo, steps, 3, warm_s=0.3)   # warmed up at its own batch, as the legs
        strong_ok[str(gb)] = ok_
        strong[str(gb)] = {"global_batch": gb, "per_rank_batch": hi - lo, "value": gb * steps / el,
                           "ms_per_step": el / steps * 1e3, "steps": steps, "truth_table_ok": ok_}
    if strong:
        line["strong"] = strong

    # every rank's identity and results (N > 1): the world the line was measured on, proven from the
    # ranks themselves — each one's device (PCI bus id, UUID) and its own truth-table / parity checks
    if world > 1:
        line["ranks"] = rank_block(dist, torch, local, backend, rank, world, truth_ok, parity, strong_ok,
                                   local_ms_per_step)
        for k_, e_ in line.get("strong", {}).items():
            e_["truth_table_ok_per_rank"] = [r["strong_truth_table_ok"].get(k_) for r in line["ranks"]["per_rank"]]

    # the host-pointer API (tfhe_amd_gate_batch_host: inputs and results in host memory, staged
    # through pinned buffers, slices of 1 024 pipelined): PCIe-inclusive, never `value`
    if world == 1 and args.host_batches not in ("none", "", "''"):
        hp, hs = {}, {}
        for s_ in args.host_batches.split(","):
            b = int(s_)
            x, y, dev, r_a, r_b, host_in = make_batch(b)
            # pinned: the caller owns page-locked arrays (T.host_empty = tfhe_amd_host_alloc), the call
            # DMAs straight from and into them; staged: ordinary (pageable) arrays, staged by the library
            pin_in = [T.host_copy(v) for v in host_in]
            modes = (("pinned", pin_in, (T.host_empty((b, 500)), T.host_empty(b)), hp),
                     ("staged", host_in, (np.zeros((b, 500), np.int32), np.zeros(b, np.int32)), hs))
            # the same batch from HBM-resident inputs, called synchronously in this leg (same clock state)
            sync_ts = []
            t_w = time.perf_counter()
            while time.perf_counter() - t_w < 0.3 or len(sync_ts) < 7:   # warmed up at this load first
                t0 = time.perf_counter()
                ctx.gate_dev(args.gate, r_a, r_b, *dev, stream=stream)
                torch.cuda.synchronize()
                sync_ts.append(time.perf_counter() - t0)
            dev_sync_ms = float(np.median(sync_ts[-5:])) * 1e3
            for mode, inp, out, dst in modes:
                # warm-up calls first: the first calls size the staging and warm the copy threads, and
                # the GPU's first touches of freshly pinned host pages are slow (the address
                # translations; r05f: 3.77 -> 3.23 ms over the first 7 pinned calls at B = 1024)
                ts = []
                for k in range(21):
                    t0 = time.perf_counter()
                    ctx.gate_host(args.gate, *inp, out=out)
                    if k >= 12:
                        ts.append(time.perf_counter() - t0)
                ms = float(np.median(ts)) * 1e3
                ok = bool(np.array_equal(K.decrypt(*out), 1 - (x & y))) if args.gate == "NAND" else None
                dst[str(b)] = {"value": b / ms * 1e3, "ms_per_call": ms, "calls": len(ts), "statistic": "median",
                               "truth_table_ok": ok, "arrays": mode,
                               "device_sync_ms_per_call": dev_sync_ms, "vs_device_sync_call": ms / dev_sync_ms,
                               "vs_device_ms_per_step": ms / line["ms_per_step"] if b == B else None}
        for d_ in (hp, hs):   # against the device path at the same batch (the headline or a `batches` leg)
            for k_, e_ in d_.items():
                dv = value if int(k_) == B else extras.get(k_, {}).get("value")
                e_["vs_device_value"] = None if not dv else e_["value"] / dv
        # `host_path` is the staged path (ordinary pageable arrays), as it was through round 4;
        # `host_path_pinned` the caller-owned page-locked arrays (round 5)
        line["host_path"] = hs
        line["host_path_pinned"] = hp

    # BASELINE configs 3-5 (circuits), every rank: config 5's rows sharded over the ranks
    if not args.no_circuits:
        line["circuits"] = circuits_leg(T, torch, ctx, K, rank, world, dist, red_dev)

    # clock under this load (rank 0 samples its own GPU; other ranks keep their GPUs busy too) and
    # the sustained fp64 ceiling: after the timed legs, whose clocks the seconds of full-power load
    # these two runs put on the chip would otherwise lower
    if not args.no_clock and fft:
        clk = sample_clock(local, main_step)
        torch.cuda.synchronize()
        if clk:
            held = FP64_PEAK_TFLOPS * clk["mhz"] / PEAK_CLOCK_MHZ
            roof["clock"] = {"gfx_mhz": clk["mhz"], "samples": clk["samples"],
                             "fp64_peak_at_clock": held, "frac_at_clock": roof["achieved"] / held}
    # the fp64 rate the chip sustains under its power limit (tfhe_amd_fp64_ceiling: register-
    # operand FMA chains on every SIMD), at the kernel's occupancy and at the best one
    if not args.no_ceiling and fft:
        ceil = {}
        for wps in (2, 8):
            tf, mhz = T.fp64_ceiling(local, wps, 2.0)
            ceil[wps] = (tf, mhz)
        roof["sustained"] = {
            "tflops_at_occupancy": ceil[2][0], "mhz_at_occupancy": ceil[2][1], "waves_per_simd": 2,
            "frac_at_occupancy": roof["achieved"] / ceil[2][0],
            "tflops_best": ceil[8][0], "mhz_best": ceil[8][1], "frac_best": roof["achieved"] / ceil[8][0],
            "note": "fp64 FMA chains on register operands on every SIMD for 2 s (no memory, no LDS): "
                    "the rate the chip holds under its power limit; k_blind_rotate_v6 runs 2 waves "
                    "per SIMD at B = 1024 (DESIGN.md 5.1)"}
    if world > 1:
        dist.barrier()

    # one process driving every visible GPU through the library (tfhe_amd_multi_gate_batch_dev:
    # device-resident shards, one key replica per device, no collective) — what a C++ host such as
    # cloud.cpp gets without torchrun; only when this single process sees several GPUs
    if world == 1 and not args.no_multi and (torch.cuda.device_count() > 1 or args.multi_devices):
        line["one_process_multi_device"] = run_multi_child(args)

    gd, gr = ctx.guard_stats()
    line["guard"] = {"max_distance": gd, "recomputed": gr, "threshold": 0.125,
                     "what": "largest rounding distance |c - rint(c)| over the sampled external-product "
                             "coefficients (one per lane and CMux step) of every bootstrap this process ran (all "
                             "legs; the 1/8 rule itself is checked on every coefficient), and the ciphertexts the "
                             "exact kernel recomputed (DESIGN.md 3.1)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(K.bk, K.ksk, rec["inputs"], rec["outputs"], args.cpu_seconds)
        parity["vs_cpu_port"] = line["cpu_baseline"]["outputs_vs_gpu"]
        line["gpu_over_cpu"] = value / line["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    K.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
