#!/usr/bin/env python3
"""From rocprofv3 --kernel-trace CSVs (one file per process): how much of each rank's all-reduce kernel
time (xg_allreduce_*) ran concurrently with its own other kernels (GEMMs, attention, ...)."""
import csv
import glob
import sys


def union_overlap(s, e, ivs):
    tot, cur = 0, s
    for a, b in ivs:
        if b <= cur:
            continue
        if a >= e:
            break
        a = max(a, cur)
        b = min(b, e)
        if b > a:
            tot += b - a
            cur = b
    return tot


files = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))
print(f"{'file':<40} {'AR kernels':>10} {'AR us':>10} {'overlapped us':>14} {'pct':>6}")
for f in files:
    rows = list(csv.DictReader(open(f)))
    ar, other = [], []
    for r in rows:
        iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        (ar if "xg_allreduce" in r["Kernel_Name"] else other).append(iv)
    other.sort()
    tot = sum(b - a for a, b in ar)
    ov = sum(union_overlap(a, b, other) for a, b in ar)
    if ar:
        print(f"{f.split('/')[-1][:40]:<40} {len(ar):>10} {tot / 1e3:>10.1f} {ov / 1e3:>14.1f} {100 * ov / max(tot, 1):>6.1f}")
