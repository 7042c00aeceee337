"""Per-kernel average time from a rocprofv3 --stats output dir: python tools/kstats.py DIR"""
import csv
import glob
import sys

for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:64]:64s} {r['Calls']:>6} {float(r['AverageNs']) / 1000:9.2f} us")
