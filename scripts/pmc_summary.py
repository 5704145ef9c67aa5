"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) into
profiles/pmc_summary.json: per-launch HBM bytes of each engine kernel.
    python scripts/pmc_summary.py <fetch_csv> <write_csv> <engine> <batch>
gfx950: FETCH_SIZE (KB) reports half the bytes of 16-B-per-lane streaming reads
(MI355X_MICROARCH.md §HBM) -> doubled; WRITE_SIZE (KB) taken as is."""
import csv, json, sys, os


def avg(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    fetch, write, engine, batch = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    f, w = avg(fetch, "FETCH_SIZE"), avg(write, "WRITE_SIZE")
    kern = {}
    for name in f:
        # the fp64 kernel is the dominant one; the exact kernel in guard mode (v4 launches whose
        # workgroups exit at once unless a ciphertext was flagged) is kept apart
        key = ("blind_rotate" if "k_blind_rotate_v6" in name else "guard" if "k_blind_rotate_v4" in name
               else "keyswitch" if "keyswitch" in name else None)
        if key is None:
            continue
        kern[key] = {"kernel": name, "fetch_kb_raw": f[name], "write_kb": w.get(name, 0.0),
                     "hbm_bytes_per_launch": (2 * f[name] + w.get(name, 0.0)) * 1024}
    out = {"engine": engine, "batch": batch, "kernels": kern,
           "source": [os.path.basename(fetch), os.path.basename(write)]}
    json.dump(out, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     "profiles", "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
