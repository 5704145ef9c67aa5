"""bench.py's JSON line against the driver's contract (the fields the round-end bench is read by):
a short GPU run with the cheap legs only, the line parsed and its fields checked, the headline
config named after BASELINE.json, the roofline's achieved rate recomputed from its own fields."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_help_runs_without_gpu():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--steps" in r.stdout and "--warmup" in r.stdout


def test_committed_pmc_summary_is_the_headlines():
    """bench.py's `roofline.traffic` comes from profiles/pmc_summary.json only when that summary is
    the headline's (this library's engine string, B = 1 024, the throughput kernel): a summary of
    another batch (a B = 1 counter pass once overwrote it) would silently null the field."""
    sys.path.insert(0, REPO)
    import bench
    import tfhe_amd as T
    s = json.load(open(os.path.join(REPO, "profiles", "pmc_summary.json")))
    assert s["batch"] == 1024 and s["engine"] == T.version(), (s["batch"], s["engine"])
    assert "k_blind_rotate_v6<2, true>" in s["kernels"]["blind_rotate"]["kernel"]
    traffic, src = bench.pmc_traffic(T.version(), 1024)
    assert traffic and traffic > 0 and src


@pytest.mark.gpu
def test_bench_line_fields():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "2",
           "--no-clock", "--no-ceiling", "--extra-batches", "none", "--strong-batch", "0", "--host-batches", "none",
           "--no-circuits", "--cpu-seconds", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = _line(r.stdout)
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert base["metric"].startswith(d["metric"])
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 2 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["config"]["batch_per_gpu"] == 1024 and "workload" in d["config"]
    # value = the batch's gates per ms_per_step
    assert abs(d["value"] - 1024 / (d["ms_per_step"] / 1e3)) / d["value"] < 1e-6
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["unit"] == "TFLOP/s" and rf["peak"] == 78.6
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert abs(rf["achieved"] - rf["flops_per_launch"] / (rf["kernel_ms"] / 1e3) / 1e12) / rf["achieved"] < 1e-6
    assert 0 < rf["kernel_ms"] < d["ms_per_step"]
    # the committed PMC summary is the headline's (test_committed_pmc_summary_is_the_headlines)
    assert rf["traffic"] and rf["traffic"] > 0 and rf["hbm"]["traffic_source"]
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0
    assert d["truth_table_ok"] is True and d["parity"]["mismatches"] == 0


@pytest.mark.gpu
def test_bench_circuits_leg_small(keyset, ctx):
    """bench.py's `circuits` leg (BASELINE configs 3-5) at a reduced matrix: every entry carries
    seconds, bootstraps/s, depth and a decrypted-correct flag, and every flag is True."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench
    import tfhe_amd as T
    out = bench.circuits_leg(T, torch, ctx, keyset, 0, 1, dist, "cpu", rows5=4, shard5=2)
    for name in ("config3_add32", "config3_add32_prefix", "config4_mul16_b256", "config5_matvec64"):
        e = out[name]
        assert e["correct"] is True, (name, e)
        assert e["seconds"] > 0 and e["bootstraps_per_s"] > 0 and e["depth"] > 0, (name, e)
    assert out["config3_add32"]["depth"] == 32 and out["config3_add32"]["bootstraps_per_instance"] == 64
    assert out["config5_matvec64"]["rows_per_rank"] == 4 and out["config5_matvec64"]["shard_of_8"]["rows"] == 2
