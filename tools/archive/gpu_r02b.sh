#!/bin/bash
# Round-2 GPU pass B: new/fixed tests, MSM A/Bs, accumulation counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02b}
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread tests/test_icicle_replay_gpu.py "tests/test_configs_full.py::test_groth16_2p24_synthetic_pk" "tests/test_msm_gpu.py::test_msm_constant_scalars_c16" > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|\] " gpurun_out/${T}_tests.log | tail -30
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|error" gpurun_out/${T}_tests.log | head -60; exit $rc; }
for s in uniform zero one wire; do timeout -k 10 120 python tools/msm_only.py --scalars $s --reps 5 || exit 1; done
for acc in prefetch noprefetch; do
  GM_MSM_ACCUM=$acc timeout -k 10 120 python tools/msm_only.py --g2 --reps 3 || exit 1
  GM_MSM_ACCUM=$acc timeout -k 10 200 python tools/msm_only.py --curve bls12377 --g2 --logn 20 --reps 3 || exit 1
done
bash tools/gpu_pmc.sh ${T}_g1 --reps 3
