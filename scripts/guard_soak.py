"""guard_soak.py — the exactness guard over many keys and millions of bootstraps.

For each of K seeded keys: R batches of B random bootsNAND through the default path (fp64 blind
rotation + guard + key switch), every output decrypted against the truth table; then the guard's
counters for that key: the ciphertexts it flagged and recomputed exactly (any coefficient of any
of the 500 CMux steps at rounding distance >= 1/8, or outside the shifter's binade) and the
largest sampled rounding distance (one coefficient per lane and step).  One JSON line per key and
a summary line.
    python scripts/guard_soak.py [--keys K] [--reps R] [--batch B]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cpu-gpu-tfhe_amd"))
import tfhe_amd as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=16)
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    tot = {"keys": 0, "bootstraps": 0, "recomputed": 0, "max_distance": 0.0, "truth_table_ok": True}
    t0 = time.time()
    for k in range(args.keys):
        K = T.SecretKeyset(seed=(7919, 104729, 1000 + k))
        c = T.Context(K.bk, K.ksk)
        try:
            c.guard_stats(reset=True)
            rng = np.random.default_rng(k)
            ok = True
            for _ in range(args.reps):
                x, y = rng.integers(0, 2, args.batch), rng.integers(0, 2, args.batch)
                out = c.gate_host("NAND", *(K.encrypt(x, rng) + K.encrypt(y, rng)))
                ok &= bool(np.array_equal(K.decrypt(*out), 1 - (x & y)))
            d, r = c.guard_stats()
        finally:
            c.close()
            K.close()
        n = args.reps * args.batch
        line = {"key": k, "bootstraps": n, "recomputed": r, "max_sampled_distance": d, "truth_table_ok": ok,
                "elapsed_s": round(time.time() - t0, 1)}
        print(json.dumps(line), flush=True)
        tot["keys"] += 1
        tot["bootstraps"] += n
        tot["recomputed"] += r
        tot["max_distance"] = max(tot["max_distance"], d)
        tot["truth_table_ok"] &= ok
    tot["cmux_steps"] = tot["bootstraps"] * 500
    tot["coefficient_roundings_checked"] = tot["cmux_steps"] * 2 * 1024
    tot["distance_samples"] = tot["cmux_steps"] * 2 * 64
    tot["engine"] = T.version()
    tot["elapsed_s"] = round(time.time() - t0, 1)
    print(json.dumps({"summary": tot}), flush=True)


if __name__ == "__main__":
    main()
