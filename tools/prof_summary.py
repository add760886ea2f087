#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats kernel_stats.csv (short names)."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("gm::", "")
    return name[:70]


def main(path):
    rows = list(csv.DictReader(open(path)))
    print("%-70s %7s %12s %12s %7s" % ("kernel", "calls", "total_ms", "avg_us", "pct"))
    for r in rows:
        print("%-70s %7s %12.3f %12.2f %7.2f" % (short(r["Name"]), r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                                 float(r["AverageNs"]) / 1e3, float(r["Percentage"])))


if __name__ == "__main__":
    main(sys.argv[1])
