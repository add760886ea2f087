#!/usr/bin/env python3
"""VALU utilisation per kernel from rocprofv3 --pmc CSV dirs (tools/gpu_pmc.sh).

  python tools/pmc_valu.py OUT.json DIR [DIR ...]

VALUBusy uses the gfx9 derived-counter formula (ROCm 7.2 ships no gfx950
section, MI355X_MICROARCH.md "rocprofv3 PMC slots"):
    SQ_ACTIVE_INST_VALU * 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs)
with 1024 SIMDs (256 CUs x 4) and GRBM_GUI_ACTIVE summed over the 8 XCDs.  It
counts 4 cycles per wave-instruction; v_mad_u64_u32 issues in ~5.1
(profiles/r01_isa_rate.txt), so the true busy fraction is at least this."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("gm::", "")
    return name.strip()


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    per[short(row["Kernel_Name"])][row["Counter_Name"]][(d, row["Dispatch_Id"])] += \
                        float(row["Counter_Value"] or 0)
    res = {}
    for k, cs in per.items():
        v = {c: sum(x.values()) / len(x) for c, x in cs.items()}
        if "SQ_ACTIVE_INST_VALU" not in v or not v.get("GRBM_GUI_ACTIVE"):
            continue
        e = {"valu_busy": round(v["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / (v["GRBM_GUI_ACTIVE"] / XCDS), 4)}
        if v.get("SQ_WAVES") and "SQ_INSTS_VALU" in v:
            e["valu_insts_per_wave"] = round(v["SQ_INSTS_VALU"] / v["SQ_WAVES"], 1)
        if v.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in v:
                    e[c.lower() + "_per_wave_cycle"] = round(v[c] / v["SQ_WAVE_CYCLES"], 4)
        res[k] = e
    res["_meta"] = {"formula": "SQ_ACTIVE_INST_VALU*4/1024/(GRBM_GUI_ACTIVE/8)", "dirs": dirs}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
