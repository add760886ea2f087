#!/bin/bash
# r05k: parity of the internal-layout NTT passes and the v4 accumulation groups
# (NTT, computeH, Groth16, PLONK / icicle replays, MSM, configs incl. 2^24), then
# same-box A/Bs: NTT GM_NTT_INT=1 vs 0, accumulation GM_MSM_ACC_V4=1 vs 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05k; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_groth16_gpu.py tests/test_plonk_replay_gpu.py tests/test_icicle_replay_gpu.py tests/test_msm_gpu.py tests/test_configs_full.py tests/test_r1cs_gpu.py tests/test_pk_io_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do
  for v in 1 0; do
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22"; do
      echo -n "int=$v $args: "; GM_NTT_INT=$v timeout -k 10 120 python3 tools/ntt_only.py $args || exit 1
    done
  done
done > $O/ntt_int_ab.txt 2>&1 || { tail -20 $O/ntt_int_ab.txt; exit 1; }
cut -c1-120 $O/ntt_int_ab.txt
bash tools/gpu_r05h.sh
