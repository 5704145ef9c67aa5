"""Average per-launch PMC values of the blind-rotation kernel from scripts/pmc_lds.sh output."""
import csv
import glob
import sys

agg = {}
for f in sorted(glob.glob(f"{sys.argv[1]}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v) / len(v):16.4g}")
