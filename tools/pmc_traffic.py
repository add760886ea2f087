#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

  python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]

Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
(16 B/lane) streaming reads, so it is doubled here; WRITE_SIZE is taken as is.
Other access widths are uncalibrated -- the JSON records the correction used.
Writes {kernel_short_name: bytes_per_launch, ...} (+ a "_meta" entry).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("gm::", "")
    return re.sub(r"<.*", "", name).strip()


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                cname = row.get("Counter_Name") or row.get("Counter") or ""
                if cname != counter:
                    continue
                k = short(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(per[k]))
                per[k].append((did, float(row.get("Counter_Value") or row.get("Value") or 0)))
    out = {}
    for k, vals in per.items():
        # sum over dimensions (XCC / agents) within one dispatch, then average dispatches
        by = defaultdict(float)
        for did, v in vals:
            by[did] += v
        out[k] = sum(by.values()) / len(by)
    return out


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        res[k] = int(2 * 1024 * fetch.get(k, 0.0) + 1024 * write.get(k, 0.0))
    res["_meta"] = {"fetch_kib": fetch, "write_kib": write,
                    "correction": "bytes = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE (gfx950 FETCH_SIZE halving "
                                  "of 16-B-per-lane streaming reads); 64-byte random gathers are tallied 1:1 "
                                  "(profiles/r05f_gather_fetch_calibration.txt), so for a gather-dominated "
                                  "kernel 1024 * FETCH_SIZE is the closer byte count"}
    s = json.dumps(res, indent=1, sort_keys=True)
    if out_path:
        with open(out_path, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
