#!/usr/bin/env python3
"""Mean SQ counter values per dispatch of each kernel from rocprofv3 --pmc csv output
(tools/debug/pmc_native.sh, pmc_tick.sh), optionally per unit (agents or envs of a dispatch).

  python tools/debug/sq_summary.py <dir> [units_per_dispatch] [kernel-substring]
"""

import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    units = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    want = sys.argv[3] if len(sys.argv) > 3 else ""
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0]
                if want in k:
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, ctrs in sorted(acc.items()):
        print(k)
        for c, v in sorted(ctrs.items()):
            m = sum(v) / len(v)
            print(f"  {c:24s} {m:16.1f}  per unit {m / units:12.2f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
