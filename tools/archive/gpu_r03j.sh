#!/bin/bash
# r03j: full -m gpu suite with the per-curve pair prefetch default (BLS12-377
# off), then BN254 G2 lane pairs without prefetch at three waves per SIMD
# (GM_MSM_PAIR_WPE=3) vs the default: G2 parity tests under it, alternated
# timings, Groth16 2^24 prove.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03j}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/${T}_tests.log)"
GM_MSM_PAIR_WPE=3 timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "g2 or G2 or True" > gpurun_out/${T}_tests_w3.log 2>&1 || { tail -30 gpurun_out/${T}_tests_w3.log; exit 1; }
echo "wpe3 msm tests: $(tail -1 gpurun_out/${T}_tests_w3.log)"
for rep in 1 2; do
  for w in def 3; do
    for args in "--g2 --logn 20 --reps 5" "--g2 --logn 20 --reps 5 --precompute"; do
      echo -n "wpe=$w $args: "
      if [ $w = 3 ]; then export GM_MSM_PAIR_WPE=3; else unset GM_MSM_PAIR_WPE; fi
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GM_MSM_PAIR_WPE
cut -c1-150 gpurun_out/${T}_ab.txt
for w in def 3 def 3; do
  if [ $w = 3 ]; then export GM_MSM_PAIR_WPE=3; else unset GM_MSM_PAIR_WPE; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$w.json 2> gpurun_out/${T}_g16_$w.err || { tail -20 gpurun_out/${T}_g16_$w.err; exit 1; }
  python3 -c "
import json; g=json.load(open('gpurun_out/${T}_g16_$w.json'))['secondary']['groth16'][0]; print('g16 wpe=$w', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
