#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace kernel_trace.csv by (kernel, grid size).

rocprofv3's kernel_stats.csv averages every launch of a kernel name, and the
bench's default run launches the G1 accumulation at several sizes (the 2^20
bench MSM, the precomputed 2^20 line, the Groth16 MSMs).  This groups the
launches by grid as well, so the bench MSM's launches have their own average;
`--last K` adds the average of the last K launches of each group (the timed
loop's launches come after the warm-up and latency ones).

  python3 tools/prof_trace_summary.py TRACE.csv[.gz] [--match NAME] [--last K]
  python3 tools/prof_trace_summary.py TRACE.csv[.gz] --match NAME --grid G --skip S --take K
      (the launches S .. S+K-1, in time order, of NAME at grid G: bench.py's timed
      loop is launches 8 .. 27 of the 2^20 accumulation grid -- 5 warm-up and 3
      latency MSMs come first; the Groth16 2^20 MSMs share the grid later.
      --grid 0 with --take: the grid of NAME's first launch, i.e. the bench MSM's)
"""
import gzip
import argparse
import csv
import re
from collections import OrderedDict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("gm::", "")[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="", help="substring of the kernel names to keep")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--grid", type=int, default=-1)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--take", type=int, default=0)
    a = ap.parse_args()
    groups = OrderedDict()
    with (gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)) as f:
        for r in csv.DictReader(f):
            name = short(r["Kernel_Name"])
            if a.match and a.match not in name:
                continue
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            groups.setdefault((name, grid), []).append((t0, t1))
    if a.grid == 0 and a.take:
        first = min(((min(ts)[0], g) for (name, g), ts in groups.items()), default=(0, 0))
        a.grid = first[1]
    if a.grid > 0:
        for (name, grid), ts in groups.items():
            if grid != a.grid:
                continue
            ts.sort()
            sel = ts[a.skip:a.skip + a.take] if a.take else ts[a.skip:]
            d = [(t1 - t0) / 1e3 for t0, t1 in sel]
            gaps = [(sel[i + 1][0] - sel[i][1]) / 1e3 for i in range(len(sel) - 1)]
            print("%s grid=%d launches %d..%d: avg %.2f us (min %.2f, max %.2f); gaps to the next launch: min %.2f us "
                  "(negative = overlap)" % (name, grid, a.skip, a.skip + len(d) - 1, sum(d) / len(d), min(d), max(d),
                                            min(gaps) if gaps else 0.0))
        return
    print("%-64s %10s %6s %12s %10s %s" % ("kernel", "grid", "calls", "total_ms", "avg_us",
                                            "avg_us_last%d" % a.last if a.last else ""))
    for (name, grid), ts in sorted(groups.items(), key=lambda kv: -sum(t1 - t0 for t0, t1 in kv[1])):
        ts.sort()
        d = [(t1 - t0) / 1e3 for t0, t1 in ts]
        line = "%-64s %10d %6d %12.3f %10.2f" % (name, grid, len(d), sum(d) / 1e3, sum(d) / len(d))
        if a.last and len(d) >= a.last:
            line += " %10.2f" % (sum(d[-a.last:]) / a.last)
        print(line)


if __name__ == "__main__":
    main()
