#!/bin/bash
# r04c: radix-4 NTT passes: NTT / computeH / Groth16 parity (incl. 2^24 all modes + the 2^24 sharded prove),
# then same-box timings radix-4 vs radix-2 (GM_NTT_R4=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04c}
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_ntt_tests.log 2>&1 || { tail -30 gpurun_out/${T}_ntt_tests.log; exit 1; }
tail -1 gpurun_out/${T}_ntt_tests.log
for rep in 1 2; do
  for v in r4 r2; do
    if [ $v = r2 ]; then export GM_NTT_R4=0; else unset GM_NTT_R4; fi
    for args in "--logn 24" "--logn 24 --coset" "--logn 20" "--curve bls12377 --logn 22"; do
      echo -n "$v: "; timeout -k 10 120 python tools/ntt_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GM_NTT_R4
cut -c1-110 gpurun_out/${T}_ab.txt
timeout -k 10 800 python -u -m pytest tests/test_configs_full.py tests/test_groth16_gpu.py tests/test_plonk_replay_gpu.py tests/test_icicle_replay_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
