#!/usr/bin/env python3
"""Median kernel time per shape from a rocprofv3 kernel trace of tools/probes/sm_trace.py.
    python tools/probes/sm_trace_parse.py <kernel_trace.csv> <sm_trace stdout>"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
shapes = [ln.split()[1:] for ln in open(sys.argv[2]) if ln.startswith("SHAPE")]
main = [r for r in rows if "smfma_kernel" in r["Kernel_Name"] or "sgemv_kernel" in r["Kernel_Name"]]
fin = [r for r in rows if "sgemv_finalize" in r["Kernel_Name"]]
per = len(main) // len(shapes)
for i, (dt, name, nbytes) in enumerate(shapes):
    ks = main[i * per:(i + 1) * per]
    us = [(int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in ks]
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    f = [(int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3 for k in fin
         if t0 <= int(k["Start_Timestamp"]) <= t1 + 10**6]
    med = statistics.median(us)
    kn = ks[0]["Kernel_Name"].split("(")[0].replace("void k8sllm::", "")
    print(f"{dt:4s} {name:8s} {med:7.1f} us {int(nbytes) / med / 1e6:5.2f} TB/s"
          + (f"  + finalize {statistics.median(f):.1f} us" if f else "") + f"  [{kn}]")
