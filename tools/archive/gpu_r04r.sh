#!/bin/bash
# r04r: tools/h2d_state.py -- which step of the 2^20 Groth16 bench section slows the
# later 2^24 host-input prove
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/h2d_state.py 2>&1 | tee gpurun_out/r04r_h2d_state.txt
