"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection.csv files.

usage: python tools/pmc_summary.py dir1 [dir2 ...]
"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mnist::", "")
            if "mnist" not in r["Kernel_Name"]:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.0f}" for c, v in sorted(cs.items())))
