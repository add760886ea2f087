#!/usr/bin/env python3
"""VALU budget of a Groth16 prove by kernel class, from a
rocprofv3 --pmc pass over tools/g16_only.py (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVES, GRBM_GUI_ACTIVE per dispatch):

  python3 tools/pmc_budget.py PMC_DIR PROVES SPAN_MS [OUT.json]

PROVES = proves the program ran (counted dispatches are divided by it), SPAN_MS
= the prove's measured wall time without the profiler.  Per class: wave-level
VALU instructions per prove, their issue cycles at the measured rates
(v_mad_u64_u32 5.12 cycles per wave64 instruction per SIMD, other VALU ~3.5,
DESIGN.md section 3; the class's mad share from the ISA where known), and the
chip time they need at 100 % issue on 1024 SIMDs at 2.4 GHz; and the measured
VALU-active cycles (SQ_ACTIVE_INST_VALU x 4 / SIMDs, the counter behind the
VALUBusy formula) as chip time.  The sums against SPAN_MS are how much of the
span the VALU work alone explains.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS, GHZ = 1024, 2.4
MAD_CYC, OTHER_CYC = 5.12, 3.5
# share of v_mad_u64_u32 among the VALU instructions (ISA / PMC)
MAD_SHARE = {"G1 accumulation": 1467 / 2340, "G2 accumulation": 1701 / 2830, "NTT passes": 162 / 310,
             # XYZZ full adds / doublings: assumed like the mixed add's mix
             "segment sums": 0.6, "fixup": 0.6, "bit-sum trees": 0.6}
CLASSES = [
    ("G1 accumulation", r"k_msm_accum_seg_ch<|k_msm_accum_seg_pf4<"),
    ("G2 accumulation", r"k_msm_accum_seg_pair"),
    ("NTT passes", r"k_ntt_pass"),
    ("fixup", r"k_msm_fixup|k_msm_fix_tree"),
    ("segment sums", r"k_msm_seg"),
    ("bit-sum trees", r"k_msm_bitsum"),
    ("digits + sort", r"k_msm_digits|k_msm_s1|k_msm_s2|k_msm_sm_|k_scan|k_expand|k_msm_sort"),
    ("computeH element-wise", r"k_poly|k_scale|k_bitrev|k_h_|k_compute_h|k_gather|k_r1cs"),
]


SETUP = r"k_batch_mul_base|k_random_scalars|k_msm_precompute|k_msm_convert_points|k_expand_points|k_gen_"


def klass(name):
    if re.search(SETUP, name):
        return None  # synthetic inputs and key upload: not per prove
    for c, pat in CLASSES:
        if re.search(pat, name):
            return c
    return "other"


def main():
    d, proves, span = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = klass(row["Kernel_Name"])
                if k is not None:
                    tot[k][row["Counter_Name"]] += float(row["Counter_Value"] or 0)
    res, sum_ms, sum_act = {}, 0.0, [0.0]
    for c, v in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0)):
        insts = v.get("SQ_INSTS_VALU", 0) / proves
        share = MAD_SHARE.get(c, 0.3)
        cyc = insts * (share * MAD_CYC + (1 - share) * OTHER_CYC)
        ms = cyc / SIMDS / (GHZ * 1e9) * 1e3
        sum_ms += ms
        # the counter the VALUBusy formula uses (4 per active VALU cycle, MI355X_MICROARCH.md "rocprofv3 PMC")
        act = v.get("SQ_ACTIVE_INST_VALU", 0) / proves * 4 / SIMDS / (GHZ * 1e9) * 1e3
        sum_act[0] += act
        res[c] = {"valu_insts_per_prove_G": round(insts / 1e9, 3), "waves_per_prove_K": round(v.get("SQ_WAVES", 0) /
                                                                                                proves / 1e3, 1),
                  "issue_ms_at_full_chip": round(ms, 2), "mad_share_assumed": round(share, 3),
                  "active_valu_ms_at_full_chip": round(act, 2)}
    res["_total"] = {"issue_ms_at_full_chip": round(sum_ms, 2), "span_ms": span,
                     "valu_issue_fraction_of_span": round(sum_ms / span, 3),
                     "active_valu_ms_at_full_chip": round(sum_act[0], 2),
                     "active_valu_fraction_of_span": round(sum_act[0] / span, 3),
                     "rates": "mad %.2f, other %.2f cycles per wave64 VALU instruction, %d SIMDs at %.1f GHz" % (
                         MAD_CYC, OTHER_CYC, SIMDS, GHZ)}
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
