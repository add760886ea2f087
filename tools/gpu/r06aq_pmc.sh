#!/bin/bash
# r06aq: VALU budget (final tree) of one 2^24 Groth16 prove per kernel class (plain and precomputed keys):
# one rocprofv3 --pmc pass each over tools/g16_only.py (2 proves), summarised by tools/pmc_budget.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for V in plain precomputed; do
  A=""; [ $V = precomputed ] && A="--precompute"
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r06aq_pmc_$V -o pmc -- python3 tools/g16_only.py --logn 24 --reps 1 $A > gpurun_out/r06aq_pmc_$V.out 2>&1 || { tail -5 gpurun_out/r06aq_pmc_$V.out; exit 1; }
  tail -1 gpurun_out/r06aq_pmc_$V.out
done
