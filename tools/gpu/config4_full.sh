#!/bin/bash
# configs[3]'s own circuit at 2^24 with a real oracle setup (opt-in test, ~8 min of host work)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
GM_TEST_CONFIG4_FULL=1 timeout -k 10 1100 python -u -m pytest tests/test_configs_full.py -m gpu -x -v -s --timeout 1080 --timeout-method thread -k squaring_chain_real_setup 2>&1 | tee gpurun_out/config4_full.log | tail -30
