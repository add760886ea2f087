#!/bin/bash
# r06h: VALU budget PMC passes over one 2^24 prove (plain / precomputed), then configs[3]'s real
# circuit at 2^24 with an oracle setup (opt-in test, ~10 min of host work)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/r06f_pmc.sh || exit 1
bash tools/gpu/config4_full.sh || exit 1
