"""Mean of each PMC counter per dispatch for kernels whose name contains a pattern.
usage: python tools/pmc_kernel.py run_counter_collection.csv PATTERN"""
import csv
import sys
from collections import defaultdict

path, pat = sys.argv[1], sys.argv[2]
tot, disp = defaultdict(float), defaultdict(set)
for r in csv.DictReader(open(path)):
    if pat in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{pat} {k}: {tot[k] / max(1, len(disp[k])):.0f} per dispatch ({len(disp[k])} dispatches)")
