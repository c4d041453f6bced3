"""Per-factorisation kernel breakdown from a rocprofv3 kernel_stats csv."""
import csv
import sys

path = sys.argv[1]
per = float(sys.argv[2]) if len(sys.argv) > 2 else 24.0
rows = list(csv.DictReader(open(path)))
tot = 0.0
for r in rows[:16]:
    ms = float(r["TotalDurationNs"]) / 1e6
    tot += ms
    print(f"{r['Name'][:40]:40s} {int(r['Calls']):7d} {ms / per:8.2f} ms/fact {float(r['AverageNs']) / 1e3:8.1f} us")
print(f"sum of listed: {tot / per:.2f} ms per factor+solve")
