#!/usr/bin/env python3
"""Average every PMC counter per kernel from rocprofv3 counter_collection CSVs under a dir.
  python tools/pmc_breakdown.py <dir> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        if want in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, ctr in acc.items():
    print(k)
    for c, v in sorted(ctr.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
