#!/usr/bin/env python3
"""Summarise tools/debug/pmc_tick_reqs.sh output: tick-kernel HBM read/write requests by size
class (TCC_EA0_RDREQ_32B/_64B/_128B, TCC_EA0_WRREQ/_64B) per dispatch, and the bytes they carry.

  python tools/pmc_reqs_summary.py gpurun_out/pmc_reqs > profiles/r02/tick_reqs.json
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d, cfg, kernel="tick_kernel"):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, cfg, "*", "*counter_collection.csv")):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if kernel in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    rd = 32 * m["TCC_EA0_RDREQ_32B"] + 64 * m["TCC_EA0_RDREQ_64B"] + 128 * m["TCC_EA0_RDREQ_128B"]
    wr = 64 * m["TCC_EA0_WRREQ_64B"] + 32 * (m["TCC_EA0_WRREQ"] - m["TCC_EA0_WRREQ_64B"])
    return {
        "dispatches": len(acc["TCC_EA0_RDREQ"]),
        "requests_per_dispatch": {k: round(v, 1) for k, v in sorted(m.items())},
        "read_bytes_by_size_class": round(rd),
        "fetch_size_bytes_x2": round(2 * 64 * m["TCC_EA0_RDREQ"]),
        "read_128B_fraction": round(m["TCC_EA0_RDREQ_128B"] / m["TCC_EA0_RDREQ"], 4),
        "write_bytes_by_size_class": round(wr),
    }


if __name__ == "__main__":
    d = sys.argv[1]
    out = {c: summarise(d, c) for c in sorted(os.listdir(d)) if os.path.isdir(os.path.join(d, c))}
    json.dump(out, sys.stdout, indent=1)
    print()
