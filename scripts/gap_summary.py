"""Launch gaps of a rocprofv3 kernel trace: per kernel name, the median
kernel duration and the median idle gap in front of it (previous kernel's end
-> its start) over the last N launches.  usage: gap_summary.py TRACE.csv [N]"""
import collections
import csv
import statistics
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1400
rows = rows[-n:]
dur, gap = collections.defaultdict(list), collections.defaultdict(list)
for (s0, e0, _), (s1, e1, k) in zip(rows, rows[1:]):
    dur[k].append(e1 - s1)
    gap[k].append(s1 - e0)
tot_d = sum(e - s for s, e, _ in rows[1:])
tot_g = sum(s1 - e0 for (_, e0, _), (s1, _, _) in zip(rows, rows[1:]))
print(f"launches {len(rows)}  kernel-sum {tot_d / 1e3:.1f} us  gap-sum {tot_g / 1e3:.1f} us  "
      f"median gap {statistics.median(s1 - e0 for (_, e0, _), (s1, _, _) in zip(rows, rows[1:])) / 1e3:.2f} us")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    print(f"{len(dur[k]):6d}  dur {statistics.median(dur[k]) / 1e3:7.2f} us  gap {statistics.median(gap[k]) / 1e3:6.2f} us  {k[:90]}")
