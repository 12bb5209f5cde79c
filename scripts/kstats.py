"""Top kernels of a rocprofv3 --stats kernel_stats.csv: share, calls, average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms, per step {tot / 1e6 / steps:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f}us "
          f"{r['Name'][:100]}")
