#!/usr/bin/env python3
"""Per-kernel averages and one step's timeline of the C5 root rehearsal from a rocprofv3 kernel
trace (tools/gpu_check_r6.sh rootprof / scale2): the kernels after the first fused-check launch
(record_check_kernel) belong to bench.py's root_loaded pass. Usage: c5_root_timeline.py <trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
first = [i for i, r in enumerate(rows) if "record_check_kernel" in r["Kernel_Name"]]
seg = rows[first[0] - 40:]
print(f"root pass: {len(first)} steps, {(seg[-1]['e'] - seg[0]['s']) / 1e6:.3f} ms traced")
agg = collections.defaultdict(lambda: [0, 0.0, set()])
for r in seg:
    a = agg[r["Kernel_Name"][:60]]
    a[0] += 1
    a[1] += (r["e"] - r["s"]) / 1e3
    a[2].add(r["Stream_Id"])
for k, (n, t, st) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:60s} n={n:5d} avg_us={t / n:8.2f} streams={sorted(st)}")
mid = first[len(first) // 2]
tc = rows[mid]["s"]
print("--- one step around a middle check launch (us from it; duration; stream)")
for r in rows:
    if tc - 300000 < r["s"] < tc + 250000:
        print(f"{(r['s'] - tc) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} st={r['Stream_Id']} {r['Kernel_Name'][:50]}")
