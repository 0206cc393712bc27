#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'total_ms':>9} {'pct':>5} {'calls':>7} {'avg_us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} {100 * float(r['TotalDurationNs']) / tot:5.1f} {r['Calls']:>7} "
          f"{float(r['AverageNs']) / 1e3:9.2f}  {r['Name'][:100]}")
print(f"all kernels: {tot / 1e6:.1f} ms")
lib = [r for r in rows if any(m in r["Name"] for m in ("Cijk_", "scaled_mm", "hipblaslt", "rocblas", "_gemm_"))]
print(f"library GEMM kernels (Cijk_ / scaled_mm / hipBLASLt / rocBLAS): {len(lib)} names, "
      f"{sum(int(r['Calls']) for r in lib)} calls, {sum(float(r['TotalDurationNs']) for r in lib) / 1e6:.1f} ms")
