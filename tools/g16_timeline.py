#!/usr/bin/env python3
"""Per-kernel timeline of the last Groth16 prove in a rocprofv3 kernel trace
(csv), grouped into phases.  Usage: tools/g16_timeline.py <prof_kernel_trace.csv> [--all]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_gather_fr" in r["Kernel_Name"]]
start = idx[-3]
t0 = int(rows[start]["Start_Timestamp"])
agg = collections.OrderedDict()
prev = t0
busy = 0
for r in rows[start:]:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    name = name.replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim::")[:60]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "--all" in sys.argv:
        print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} gap {(s - prev) / 1e6:7.3f} {name}")
    a = agg.setdefault(name, [0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e6
    busy += e - s
    prev = e
print("span %.3f ms, kernels busy %.3f ms" % ((prev - t0) / 1e6, busy / 1e6))
for k, (cnt, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{ms:9.3f} ms {cnt:4d}x  {k}")
