"""Average every PMC counter per kernel (short name) over the counter_collection CSVs of a directory tree."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "?")
            short = name.split("(")[0].split("<")[0][-60:]
            if "mgemm" in name or "pgemm" in name:
                short = name.split("(")[0].split("::")[-1][:90]
            acc[short][r.get("Counter_Name", "?")].append(float(r.get("Counter_Value", 0) or 0))
for k, d in sorted(acc.items()):
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):14.1f}  (n={len(v)})")
