"""Kernel statistics (rocprofv3 --kernel-trace --stats) from a rocpd SQLite
database: per kernel name calls, total / average / min / max duration (ns) and
share of GPU time, written as CSV (the columns of rocprofv3's
kernel_stats.csv). usage: python tools/prof_stats.py results.db out.csv"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute(
    "select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
    "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = {}
for name, dur in rows:
    a = agg.setdefault(name, [0, 0, None, 0])
    a[0] += 1
    a[1] += dur
    a[2] = dur if a[2] is None else min(a[2], dur)
    a[3] = max(a[3], dur)
total = sum(a[1] for a in agg.values()) or 1
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([name, a[0], a[1], a[1] / a[0], 100.0 * a[1] / total, a[2], a[3]])
print("wrote", out, len(agg), "kernels")
