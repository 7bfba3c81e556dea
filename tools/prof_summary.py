"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv (diagnostic)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
tot = sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e3
print(f"total {tot:.1f} us/step")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:8.1f} us/step  n={int(r['Calls']) / steps:5.1f} "
          f"avg={float(r['AverageNs']) / 1e3:7.1f}  {r['Name'][:100]}")
