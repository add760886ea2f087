#!/usr/bin/env python3
"""Per-kernel timeline of the last Groth16 prove in a rocprofv3 kernel trace
(csv), grouped into phases.  Usage: tools/g16_timeline.py <prof_kernel_trace.csv> [--all]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last prove starts with its first digit kernel (the shared wire plan's, or
# a compaction gather when the key has no shared plan); an R1CS evaluation
# queued just before it belongs to it too
names = [r["Kernel_Name"] for r in rows]
dig = [i for i, n in enumerate(names) if "k_msm_digits" in n]
gat = [i for i, n in enumerate(names) if "k_gather_fr" in n]
if gat and gat[-1] > dig[-2]:
    start = gat[-3] if len(gat) >= 3 else gat[0]
else:
    start = dig[-2]
ev = [i for i, n in enumerate(names) if "k_r1cs_eval" in n and i < start]
if ev and int(rows[start]["Start_Timestamp"]) - int(rows[ev[-1]]["Start_Timestamp"]) < 5_000_000:
    start = ev[-1]
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
