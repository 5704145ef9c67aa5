"""Reproduce bench.py's roofline from a rocprofv3 run of the SAME command:
the blind-rotation launches of the headline's timed steps (its launches W .. W+K-1 in dispatch
order: the bench runs W warm-up steps, then K timed ones, before any other leg), their mean
duration, the --stats average of the kernel over every launch of the run, and the run's own bench
line (ms_per_step, kernel_ms from HIP events, frac) side by side.
    python scripts/trace_mean.py <kernel_trace.csv> <kernel_stats.csv> <bench_json_line_file> [steps] [warmup]"""
import csv
import json
import sys

FLOPS_PER_BOOTSTRAP = 500 * 198656
FLOPS10_PER_BOOTSTRAP = 500 * 173568
PEAK = 78.6


def is_headline_br(name):
    """the one-ciphertext-per-workgroup fp64 kernel of the headline (k_blind_rotate_v6<...>), not the
    paired / four-wave / circuit-row / debug forms"""
    return "k_blind_rotate_v6<" in name and "v6p" not in name and "v6_rows" not in name and "v6_debug" not in name


def main():
    trace, stats, bench = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    line = None
    for ln in open(bench):
        if ln.startswith("{"):
            line = json.loads(ln)
    B = line["config"]["batch_per_gpu"]
    rows = [r for r in csv.DictReader(open(trace)) if is_headline_br(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    timed = durs[warm:warm + steps]
    st = [r for r in csv.DictReader(open(stats)) if is_headline_br(r["Name"])]
    avg_timed = sum(timed) / len(timed) / 1e6
    out = {"kernel": st[0]["Name"] if st else "k_blind_rotate_v6", "batch": B, "launches_in_run": len(durs),
           "stats_average_ms": float(st[0]["AverageNs"]) / 1e6 if st else None,
           "stats_calls": int(st[0]["Calls"]) if st else None,
           "trace_mean_timed_ms": avg_timed, "timed_launches": len(timed), "timed_launch_index": [warm, warm + steps],
           "trace_min_timed_ms": min(timed) / 1e6, "trace_max_timed_ms": max(timed) / 1e6,
           "bench_ms_per_step": line["ms_per_step"], "bench_kernel_ms": line["roofline"]["kernel_ms"],
           "bench_frac": line["roofline"]["frac"], "bench_value": line["value"]}
    for k, ms in (("stats_average_ms", out["stats_average_ms"]), ("trace_mean_timed_ms", avg_timed)):
        if ms:
            out["frac_from_" + k] = B * FLOPS_PER_BOOTSTRAP / (ms * 1e-3) / 1e12 / PEAK
            out["frac10_from_" + k] = B * FLOPS10_PER_BOOTSTRAP / (ms * 1e-3) / 1e12 / PEAK
    out["timed_trace_vs_bench_kernel_ms"] = avg_timed / out["bench_kernel_ms"] - 1
    out["frac_from_trace_vs_bench_frac"] = out["frac_from_trace_mean_timed_ms"] / out["bench_frac"] - 1
    out["stats_below_ms_per_step"] = bool(out["stats_average_ms"] and out["stats_average_ms"] < line["ms_per_step"])
    out["timed_trace_below_ms_per_step"] = avg_timed < line["ms_per_step"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
