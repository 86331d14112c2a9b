"""Top kernels of a rocprofv3 --stats kernel_stats.csv: name, calls, average ms."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs']) / 1e6:.3f}")
