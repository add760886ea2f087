#!/usr/bin/env python3
"""Merged copy + kernel timeline of the last host-input Groth16 prove in a rocprofv3
trace (--kernel-trace --memory-copy-trace, csv).  H2D copies are coalesced into runs
(gaps < 0.2 ms), kernels into phases by name; times in ms relative to the first H2D
copy of the last prove (a gap > 20 ms between copies separates proves).
Usage: tools/g16_copy_timeline.py <kernel_trace.csv> <memory_copy_trace.csv>"""
import csv
import sys

kern = list(csv.DictReader(open(sys.argv[1])))
cps = list(csv.DictReader(open(sys.argv[2])))
h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cps
             if r.get("Direction", "").endswith("HOST_TO_DEVICE") or "HOST_TO_DEVICE" in r.get("Kind", ""))
# the last prove's copies: after the last gap > 20 ms
start = 0
for i in range(1, len(h2d)):
    if h2d[i][0] - h2d[i - 1][1] > 20_000_000:
        start = i
h2d = h2d[start:]
t0 = h2d[0][0]
runs = []
for s, e in h2d:
    if runs and s - runs[-1][1] < 200_000:
        runs[-1][1] = max(runs[-1][1], e)
        runs[-1][2] += e - s
    else:
        runs.append([s, e, e - s])
ev = [((s - t0) / 1e6, (e - t0) / 1e6, "H2D run (busy %.2f ms)" % (b / 1e6)) for s, e, b in runs]
phase = {}
for r in kern:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 - 5_000_000:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gm::", "")
    key = name.split("<")[0]
    p = phase.setdefault(key, [s, e, 0.0, 0])
    p[0], p[1] = min(p[0], s), max(p[1], e)
    p[2] += (e - s) / 1e6
    p[3] += 1
for k, (s, e, busy, cnt) in phase.items():
    ev.append(((s - t0) / 1e6, (e - t0) / 1e6, "%s x%d (kernel time %.2f ms)" % (k, cnt, busy)))
ev.sort()
end = max(e for _, e, _ in ev)
print("last prove: %.2f ms from the first H2D copy to the last kernel end" % end)
for s, e, what in ev:
    print("%9.3f %9.3f  %s" % (s, e, what))
