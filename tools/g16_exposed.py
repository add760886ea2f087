#!/usr/bin/env python3
"""Where a Groth16 prove's span goes, from a rocprofv3 kernel trace of
tools/g16_only.py: the last prove's window (from its first digit / gather kernel
to its last kernel), split into time covered by VALU-heavy kernels
(accumulations, NTT passes, reductions) and time when only the sort / digit /
copy kernels -- or nothing -- run.

  python3 tools/g16_exposed.py TRACE.csv[.gz]
"""
import csv
import gzip
import re
import sys

HEAVY = r"k_msm_accum|k_ntt_pass|k_msm_seg|k_msm_fixup|k_msm_bitsum|k_msm_fix_tree"


def main():
    p = sys.argv[1]
    with (gzip.open(p, "rt") if p.endswith(".gz") else open(p)) as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"])
                 .replace("void ", "").replace("gm::", "")) for r in csv.DictReader(f)]
    rows.sort()
    # the last prove: from the second-to-last wire-plan digit kernel group
    dig = [i for i, r in enumerate(rows) if "k_msm_digits" in r[2]]
    # each prove runs two plans (wires, Z): the last prove starts at dig[-2]
    start = dig[-2]
    win = rows[start:]
    t0 = win[0][0]
    t1 = max(e for _, e, _ in win)

    def union(iv):
        iv = sorted(iv)
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if cs is not None:
            tot += ce - cs
        return tot

    heavy = union([(s, e) for s, e, n in win if re.search(HEAVY, n)])
    anyk = union([(s, e) for s, e, n in win])
    span = t1 - t0
    print("last prove window %.2f ms: heavy kernels cover %.2f ms, any kernel %.2f ms; only light kernels %.2f ms, "
          "nothing %.2f ms" % (span / 1e6, heavy / 1e6, anyk / 1e6, (anyk - heavy) / 1e6, (span - anyk) / 1e6))
    # light-only stretches longer than 0.2 ms, with what runs in them
    ev = sorted(set([t0, t1] + [s for s, _, _ in win] + [e for _, e, _ in win]))
    cur = None
    for a, b in zip(ev, ev[1:]):
        act = [n for s, e, n in win if s < b and e > a]
        light = bool(act) and not any(re.search(HEAVY, n) for n in act)
        key = tuple(sorted(set(act))) if light else None
        if key and cur and cur[2] == key:
            cur[1] = b
            continue
        if cur and cur[1] - cur[0] > 200000:
            print("  %8.2f - %8.2f ms light: %s" % ((cur[0] - t0) / 1e6, (cur[1] - t0) / 1e6, ", ".join(cur[2])[:150]))
        cur = [a, b, key] if key else None
    if cur and cur[1] - cur[0] > 200000:
        print("  %8.2f - %8.2f ms light: %s" % ((cur[0] - t0) / 1e6, (cur[1] - t0) / 1e6, ", ".join(cur[2])[:150]))


if __name__ == "__main__":
    main()
