#!/bin/bash
# r04af: growing bounds in the DIT passes (GM_NTT_GROW bit 1, default on): parity over
# every NTT / computeH consumer, then same-box A/B against DIF-only growth (GM_NTT_GROW=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04af}
timeout -k 10 900 python -u -m pytest tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_configs_full.py tests/test_groth16_gpu.py tests/test_icicle_replay_gpu.py tests/test_plonk_replay_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2 3; do
  for g in 3 1; do
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22"; do
      echo -n "grow=$g $args: "; GM_NTT_GROW=$g timeout -k 10 120 python3 tools/ntt_only.py $args || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_ab.txt | cut -c1-150
for g in 3 1; do
  GM_NTT_GROW=$g timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --g16-logn 24 --g16-plain 24 --msm-extra 0 --ntt-logn 24 > gpurun_out/${T}_g16_$g.json 2> gpurun_out/${T}_g16_$g.err || { tail -20 gpurun_out/${T}_g16_$g.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g16_$g.json'))['secondary']; print('grow=$g ntt', d['ntt']['ms_per_transform'])
for g in d['groth16']: print('grow=$g g16 2^%d' % g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'])" | tee -a gpurun_out/${T}_ab.txt
done
