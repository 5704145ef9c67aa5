"""Summarise the rocprofv3 --pmc passes of one profile_round.sh session (each pass its own run of
the same bench command) into profiles/pmc_summary.json: per-launch counters of the engine's
kernels over the headline's timed launches only (dispatch order: W warm-up steps, then K timed
ones, each step = blind rotation + guard launch + key switch), HBM bytes per launch, and the
blind rotation's per-wave-step instruction counts (B ciphertexts x 2 waves x 500 CMux steps).
    python scripts/pmc_summary.py <pass_dir> <engine> <batch> [steps] [warmup] [tag]
(PMC_SUMMARY_OUT=<path> writes elsewhere, e.g. an A/B variant's summary)
gfx950: FETCH_SIZE (KB) reports half the bytes of 16-B-per-lane streaming reads
(MI355X_MICROARCH.md §HBM) -> doubled; WRITE_SIZE (KB) taken as is."""
import csv
import glob
import json
import os
import sys

KINDS = (("blind_rotate", lambda n: ("k_blind_rotate_v6<" in n and "v6p" not in n and "v6_rows" not in n)
                          or "k_blind_rotate_v10<" in n),
         ("guard", lambda n: "k_blind_rotate_v4<" in n),
         ("keyswitch", lambda n: "k_keyswitch" in n))


def launches(path):
    """{kind: [(dispatch, kernel name, {counter: value})]} in dispatch order"""
    by = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        e = by.setdefault(d, {"name": r["Kernel_Name"], "c": {}})
        e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {}
    for d in sorted(by):
        for kind, pred in KINDS:
            if pred(by[d]["name"]):
                out.setdefault(kind, []).append((d, by[d]["name"], by[d]["c"]))
    return out


def main():
    pdir, engine, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    tag = sys.argv[6] if len(sys.argv) > 6 else os.path.basename(os.path.normpath(pdir))
    counters, names, sources = {}, {}, []
    for f in sorted(glob.glob(os.path.join(pdir, "*", "**", "*counter_collection.csv"), recursive=True)):
        sources.append(os.path.relpath(f, pdir))
        for kind, ls in launches(f).items():
            sel = ls[warm:warm + steps]
            if not sel:
                continue
            names[kind] = sel[0][1]
            acc = counters.setdefault(kind, {})
            for _, _, c in sel:
                for k, v in c.items():
                    acc.setdefault(k, []).append(v)
    kern = {}
    for kind, acc in counters.items():
        avg = {k: sum(v) / len(v) for k, v in acc.items()}
        e = {"kernel": names[kind], "launches_averaged": max(len(v) for v in acc.values()), "per_launch": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["fetch_kb_raw"] = avg["FETCH_SIZE"]
            e["write_kb"] = avg["WRITE_SIZE"]
            e["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        if kind == "blind_rotate":
            ws = batch * 2 * 500     # wave-steps per launch
            e["per_wave_step"] = {k: avg[k] / ws for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD")
                                  if k in avg}
            if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
                e["wait_inst_any_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_INST_LDS" in avg and "SQ_WAVE_CYCLES" in avg:
                e["wait_inst_lds_frac"] = avg["SQ_WAIT_INST_LDS"] / avg["SQ_WAVE_CYCLES"]
        kern[kind] = e
    out = {"engine": engine, "batch": batch, "launch_selection": f"headline timed launches [{warm}, {warm + steps})",
           "kernels": kern, "source": tag, "passes": sources}
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.environ.get("PMC_SUMMARY_OUT") or os.path.join(repo, "profiles", "pmc_summary.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
