#!/bin/bash
# r04j + r04k in one call: bench MSM-loop kernel trace, then the two-stream Groth16 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/archive/gpu_r04j.sh && bash tools/archive/gpu_r04k.sh
