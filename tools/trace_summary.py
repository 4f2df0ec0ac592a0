#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, with the
early-exit launches split off.

The device-resident Krylov cycles enqueue a restart cycle's launches ahead;
once a cycle stops (tolerance or the 5000-step cap) the launches still queued
return at once (k_sell_spmv, k_sstep_block check the cycle's stop flag first).
Their ~1 us durations would pull a kernel's average far below what a working
launch takes, so a launch shorter than `frac` x the kernel's median counts as
an early exit and the roofline averages use the others.

usage: trace_summary.py run_kernel_trace.csv out.json [command] [frac=0.3]
out.json: {"kernels": {name: {calls, full_calls, early_exit_calls,
avg_ns_full, median_ns, min_ns_full, max_ns}}, ...}"""
import csv
import json
import statistics
import sys


def summarise(path, frac=0.3):
    durs = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            durs.setdefault(r["Kernel_Name"], []).append(d)
    out = {}
    for name, v in durs.items():
        med = statistics.median(v)
        full = [x for x in v if x >= frac * med]
        out[name] = {"calls": len(v), "full_calls": len(full), "early_exit_calls": len(v) - len(full),
                     "avg_ns_full": sum(full) / len(full), "median_ns": med,
                     "min_ns_full": min(full), "max_ns": max(v), "avg_ns_all": sum(v) / len(v)}
    return out


def lookup(summary, key):
    """The entry whose kernel name contains `key` (None if absent or ambiguous)."""
    hits = [v for k, v in summary["kernels"].items() if key in k]
    return hits[0] if len(hits) == 1 else None


def main():
    path, out = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    frac = float(sys.argv[4]) if len(sys.argv) > 4 else 0.3
    res = {"command": cmd, "source": path,
           "early_exit_rule": f"duration < {frac} x the kernel's median",
           "kernels": summarise(path, frac)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out, len(res["kernels"]), "kernels")


if __name__ == "__main__":
    main()
