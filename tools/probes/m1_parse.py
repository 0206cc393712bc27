#!/usr/bin/env python3
"""Median GEMV vs sgemv kernel time per shape from a kernel trace of tools/probes/m1_trace.py."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
shapes = [ln.split()[1:] for ln in open(sys.argv[2]) if ln.startswith("SHAPE")]
ks = [r for r in rows if any(s in r["Kernel_Name"] for s in ("gemv_kernel", "smfma_kernel", "sgemv_"))]
per = len(ks) // len(shapes)
for i, (name, nbytes) in enumerate(shapes):
    grp = ks[i * per:(i + 1) * per]
    gv = [(int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in grp if "gemv_kernel" in k["Kernel_Name"]]
    sm = [(int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in grp if "smfma" in k["Kernel_Name"]]
    fin = [(int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in grp if "finalize" in k["Kernel_Name"]]
    g, s = statistics.median(gv) if gv else float("nan"), statistics.median(sm) if sm else float("nan")
    print(f"{name:16s} gemv {g:7.1f} us ({int(nbytes) / g / 1e6:4.2f} TB/s)   sgemv-mfma {s:7.1f} us "
          f"({int(nbytes) / s / 1e6:4.2f} TB/s){'  (+ gemv split reduce)' if fin else ''}")
