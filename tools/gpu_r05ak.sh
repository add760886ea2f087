#!/bin/bash
# r05ak: the chained three-wave BN254 pair kernel as default: MSM / Groth16 / configs GPU tests, G2 2^20 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ak; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_configs_full.py tests/test_golden_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/msm_only.py --g2 --logn 20 --reps 5
