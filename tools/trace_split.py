"""Kernel statistics of the refine-5 part of a bench profile: the dispatches of a
rocprofv3 kernel trace (run_kernel_trace.csv) that start before the converging
refine-3 leg's first Schur SpMV (the leg runs after the timed steps), written in
the columns of rocprofv3's kernel_stats.csv.
usage: python tools/trace_split.py run_kernel_trace.csv out.csv [r3_spmv_grid]"""
import csv
import sys

src, out = sys.argv[1], sys.argv[2]
r3_grid = sys.argv[3] if len(sys.argv) > 3 else "14080"
rows = list(csv.DictReader(open(src)))
cut = min((int(r["Start_Timestamp"]) for r in rows
           if "k_sell_spmv" in r["Kernel_Name"] and r["Grid_Size_X"] == r3_grid), default=None)
agg = {}
for r in rows:
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if cut is not None and t0 >= cut:
        continue
    a = agg.setdefault(r["Kernel_Name"], [0, 0, None, 0])
    a[0] += 1
    a[1] += t1 - t0
    a[2] = t1 - t0 if a[2] is None else min(a[2], t1 - t0)
    a[3] = max(a[3], t1 - t0)
total = sum(a[1] for a in agg.values()) or 1
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([name, a[0], a[1], a[1] / a[0], 100.0 * a[1] / total, a[2], a[3]])
print("wrote", out, len(agg), "kernels", "cut at", cut)
