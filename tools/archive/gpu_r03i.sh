#!/bin/bash
# r03i: G2 lane-pair accumulation without the point prefetch (GM_MSM_PAIR_PF=0):
# G2 MSM parity tests under it, then alternated timings vs the default
# (BN254 G2 2^20 plain / precomputed, BLS12-377 G2 2^22, Groth16 2^24 prove).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03i}
GM_MSM_PAIR_PF=0 timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests_pf0.log 2>&1 || { tail -30 gpurun_out/${T}_tests_pf0.log; exit 1; }
echo "pf0 tests: $(tail -1 gpurun_out/${T}_tests_pf0.log)"
for rep in 1 2; do
  for pf in 1 0; do
    for args in "--g2 --logn 20 --reps 5" "--g2 --logn 20 --reps 5 --precompute" "--curve bls12377 --g2 --logn 22 --reps 2"; do
      echo -n "pf=$pf $args: "
      GM_MSM_PAIR_PF=$pf timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
cut -c1-150 gpurun_out/${T}_ab.txt
for pf in 1 0 1 0; do
  GM_MSM_PAIR_PF=$pf timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$pf.json 2> gpurun_out/${T}_g16_$pf.err || { tail -20 gpurun_out/${T}_g16_$pf.err; exit 1; }
  python3 -c "
import json; g=json.load(open('gpurun_out/${T}_g16_$pf.json'))['secondary']['groth16'][0]; print('g16 pf=$pf', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
