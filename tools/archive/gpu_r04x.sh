#!/bin/bash
# r04x: VALU counters of the final NTT kernels (DIF three waves with the twiddle
# prefetch, DIT four waves; one mad chain per product) at 2^24.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04x}
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_ntt_pmc_valu.json gpurun_out/${T}_ntt_pmc1 gpurun_out/${T}_ntt_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_ntt_pmc_valu.json')); print({k: v for k, v in d.items() if 'ntt' in k})"
grep -A16 "^k_ntt_pass4" gpurun_out/${T}_ntt_pmc_summary.txt | grep -E "k_ntt|SQ_INSTS_VALU|SQ_WAVES |SQ_INSTS_LDS|SQ_WAIT_ANY |SQ_WAVE_CYCLES"
