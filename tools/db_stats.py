"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 results .db:
  python tools/db_stats.py gpurun_out/TAG_prof/run_results.db profiles/TAG_kernel_stats.csv"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                   "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
acc = defaultdict(list)
for name, dur in rows:
    acc[name].append(dur)
total = sum(sum(v) for v in acc.values())
out = []
for name, v in acc.items():
    out.append([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / total, 2), min(v), max(v),
                statistics.pstdev(v)])
out.sort(key=lambda r: -r[2])
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    w.writerows(out)
for r in out[:8]:
    print(f"{r[0][:70]:70s} calls={r[1]:4d} avg={r[3]/1e6:.4f} ms  {r[4]}%")
