"""Summarise a rocprofv3 ``*_kernel_stats.csv``: one line per kernel (share, total ms, calls, mean us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}% {float(r['TotalDurationNs'])/1e6:9.1f}ms {int(r['Calls']):6d} "
          f"{float(r['AverageNs'])/1e3:9.1f}us {r['Name'][:110]}")
print(f"total {tot/1e6:.1f} ms")
