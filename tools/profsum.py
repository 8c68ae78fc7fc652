import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:8.3f} tot%={100*float(r['TotalDurationNs'])/tot:5.1f}")
print("total ms", tot/1e6)
