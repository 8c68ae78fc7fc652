"""Average duration (µs) and call count of the kernels whose names contain any of the given
substrings, from a rocprofv3 --stats directory. usage: python tools/kstats.py STATS_DIR SUBSTR..."""
import csv
import glob
import sys

path = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True))[0]
for r in csv.DictReader(open(path)):
    if any(s in r["Name"] for s in sys.argv[2:]):
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1000:8.3f} us")
