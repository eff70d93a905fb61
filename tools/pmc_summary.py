#!/usr/bin/env python3
"""Summarise rocprofv3 output of profiles/run_rocprof.sh into one JSON per config.

Per kernel: dispatch count and mean duration (kernel trace), FETCH_SIZE / WRITE_SIZE per dispatch
(separate --pmc passes; the median, which is the steady state: the mean also counts the few
launches that write every obs row in full -- the first launch into a bound buffer, the resets --
and is reported beside it) and the HBM bytes per dispatch corrected as
MI355X_MICROARCH.md §HBM prescribes: rocprofv3 reports both counters in KiB; on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (doubled here), WRITE_SIZE is exact
for 16-B-per-lane stores.

  python tools/pmc_summary.py <prof_dir/cfg> > pmc.json
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern):
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path, newline="") as f:
            yield from csv.DictReader(f)


def _short(name):
    """'void nmmo::tick_kernel<15u>(nmmo::DevState, ...)' -> 'tick_kernel' (all system-set
    specialisations of a kernel are one entry: a bench run launches only one of them)."""
    name = name.split("(")[0].split("<")[0]
    name = name.split("::")[-1].strip()
    return name[:-3] if name.endswith("_w8") else name  # occupancy variant of the same kernel


def summarise(d):
    out = defaultdict(dict)
    for r in _rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        k = _short(r["Name"])
        out[k]["dispatches"] = int(r["Calls"])
        out[k]["avg_ns"] = float(r["AverageNs"])
    # dispatches that ran alone vs while another dispatch of the same kernel ran (bench.py
    # --batches > 1 overlaps the batches' streams; its roofline times launches alone)
    spans = defaultdict(list)
    for r in _rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        spans[_short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k, sp in spans.items():
        sp.sort()
        solo, over = [], []
        for i, (a, b) in enumerate(sp):
            hit = (i > 0 and max(e for _, e in sp[max(0, i - 8):i]) > a) or (i + 1 < len(sp) and sp[i + 1][0] < b)
            (over if hit else solo).append(b - a)
        out[k]["solo_dispatches"] = len(solo)
        out[k]["solo_avg_ns"] = round(sum(solo) / len(solo), 1) if solo else None
        out[k]["overlapped_dispatches"] = len(over)
        out[k]["overlapped_avg_ns"] = round(sum(over) / len(over), 1) if over else None
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        acc = defaultdict(list)
        for r in _rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if r.get("Counter_Name") == ctr:
                acc[_short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            sv = sorted(v)
            med = sv[len(sv) // 2] if len(sv) % 2 else (sv[len(sv) // 2 - 1] + sv[len(sv) // 2]) / 2
            out[k][ctr.lower() + "_kib_per_dispatch"] = med
            out[k][ctr.lower() + "_kib_mean"] = sum(v) / len(v)
            out[k][ctr.lower() + "_dispatches"] = len(v)
    for k, v in out.items():
        if "fetch_size_kib_per_dispatch" in v and "write_size_kib_per_dispatch" in v:
            v["hbm_bytes_per_dispatch"] = round(
                2 * v["fetch_size_kib_per_dispatch"] * 1024 + v["write_size_kib_per_dispatch"] * 1024)
    return dict(out)


if __name__ == "__main__":
    d = sys.argv[1]
    res = {"kernels": summarise(d)}
    bj = os.path.join(d, "bench.json")
    if os.path.exists(bj):
        lines = [ln for ln in open(bj) if ln.strip().startswith("{")]
        if lines:
            res["bench"] = json.loads(lines[-1])
    json.dump(res, sys.stdout, indent=1)
    print()
