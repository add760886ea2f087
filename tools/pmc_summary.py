#!/usr/bin/env python3
"""Per-kernel average counter values per dispatch from rocprofv3 --pmc CSV dirs.

  python tools/pmc_summary.py DIR [DIR ...]
Counter values are summed over the dimensions of one dispatch (XCDs / SEs) and
averaged over dispatches of the same kernel.  Derived: VALU instructions per
wave, VALU-active fraction of wave cycles, issue-stall fraction."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("gm::", "")
    return name.strip()[:90]


def main():
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", ""))
                    c = row.get("Counter_Name", "")
                    did = (d, row.get("Dispatch_Id", ""))
                    per[k][c][did] += float(row.get("Counter_Value") or 0)
    for k in sorted(per):
        vals = {c: sum(v.values()) / len(v) for c, v in per[k].items()}
        print(k)
        for c in sorted(vals):
            print("   %-26s %16.1f" % (c, vals[c]))
        w = vals.get("SQ_WAVES")
        if w and "SQ_INSTS_VALU" in vals:
            print("   %-26s %16.1f" % ("valu_insts_per_wave", vals["SQ_INSTS_VALU"] / w))
        if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"]:
            wc = vals["SQ_WAVE_CYCLES"]
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in vals:
                    print("   %-26s %16.3f" % (c + "/WAVE_CYC", vals[c] / wc))


if __name__ == "__main__":
    main()
