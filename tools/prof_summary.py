import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0
for r in rows[:12]:
    a = float(r['AverageNs']) / 1000
    print(f"{r['Name'][:62]:62s} calls={r['Calls']:>6s} avg_us={a:8.2f} pct={float(r['Percentage']):6.2f}")
