"""Reproduce bench.py's roofline from a rocprofv3 run of the same command:
mean duration of the dominant kernel over ALL its launches (what --stats averages) and over the
last `steps` launches (the bench's timed region, after its warm-up), next to the bench line's
own kernel_ms from HIP events.
    python scripts/trace_mean.py <kernel_trace.csv> <kernel_stats.csv> <bench_json_line_file> [steps]"""
import csv
import json
import sys

FLOPS_PER_BOOTSTRAP = 500 * 198656
FLOPS10_PER_BOOTSTRAP = 500 * 173568
PEAK = 78.6


def main():
    trace, stats, bench = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    line = None
    for ln in open(bench):
        if ln.startswith("{"):
            line = json.loads(ln)
    B = line["config"]["batch_per_gpu"]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))
            if "k_blind_rotate_v6" in r["Kernel_Name"]]
    st = [r for r in csv.DictReader(open(stats)) if "k_blind_rotate_v6" in r["Name"]]
    avg_all = sum(durs) / len(durs) / 1e6
    tail = durs[-steps:]
    avg_tail = sum(tail) / len(tail) / 1e6
    out = {"kernel": "k_blind_rotate_v6", "batch": B, "launches": len(durs),
           "stats_average_ms": float(st[0]["AverageNs"]) / 1e6 if st else None,
           "trace_mean_all_ms": avg_all, "trace_mean_timed_ms": avg_tail, "timed_launches": len(tail),
           "bench_kernel_ms": line["roofline"]["kernel_ms"],
           "bench_frac": line["roofline"]["frac"]}
    for k, ms in (("stats_average_ms", out["stats_average_ms"]), ("trace_mean_timed_ms", avg_tail)):
        if ms:
            out["frac_from_" + k] = B * FLOPS_PER_BOOTSTRAP / (ms * 1e-3) / 1e12 / PEAK
            out["frac10_from_" + k] = B * FLOPS10_PER_BOOTSTRAP / (ms * 1e-3) / 1e12 / PEAK
    out["stats_vs_bench"] = out["stats_average_ms"] / out["bench_kernel_ms"] - 1 if out["stats_average_ms"] else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
