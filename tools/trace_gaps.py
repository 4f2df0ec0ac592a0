"""Per-kernel average duration and the average idle gap before each kernel
(previous kernel end -> this start, same queue) from a rocpd database.
usage: python tools/trace_gaps.py results.db [name-filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
agg = {}
prev_end = None
for name, st, en in rows:
    short = name.split("(")[0].replace("_ZN3dcp12_GLOBAL__N_1", "")[:60]
    a = agg.setdefault(short, [0, 0, 0])
    a[0] += 1
    a[1] += en - st
    if prev_end is not None:
        a[2] += max(0, st - prev_end)
    prev_end = en
for k, (n, dur, gap) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    print(f"{n:8d} {dur / n / 1e3:9.2f} us  gap-before {gap / n / 1e3:8.2f} us  {k}")
