#!/usr/bin/env python3
"""Overlap of the bench's pipelined MSMs in a rocprofv3 kernel trace (csv): for
the last K accumulation launches, the span between consecutive accumulation
starts, the busy union of every kernel in that window and the sum of their
durations, plus the last MSM's kernels in start order.
Usage: tools/msm_timeline.py <kernel_trace.csv> [K]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:48])
            for r in rows)
acc = [i for i, (s, e, n) in enumerate(iv) if "k_msm_accum_seg" in n]
acc = acc[-(K + 1):]
t_lo, t_hi = iv[acc[0]][0], iv[acc[-1]][0]
win = [(s, e, n) for s, e, n in iv if s >= t_lo and s < t_hi]
union, cur_s, cur_e = 0, None, None
for s, e, n in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
tot = sum(e - s for s, e, n in win)
accsum = sum(iv[i][1] - iv[i][0] for i in acc[:-1])
print("%d MSMs: %.3f ms per MSM (accumulation start to start), busy union %.3f, kernel sum %.3f, accumulation %.3f"
      % (len(acc) - 1, (t_hi - t_lo) / 1e6 / (len(acc) - 1), union / 1e6 / (len(acc) - 1), tot / 1e6 / (len(acc) - 1),
         accsum / 1e6 / (len(acc) - 1)))
a0 = iv[acc[-2]][0]
for s, e, n in iv:
    if a0 - 1_500_000 <= s < iv[acc[-1]][0]:
        print("%9.3f %9.3f %8.3f  %s" % ((s - a0) / 1e6, (e - a0) / 1e6, (e - s) / 1e6, n))
