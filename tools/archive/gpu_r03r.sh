#!/bin/bash
# r03r: G1 accumulation with the next key / value prefetched (GM_MSM_ACCUM=idx)
# vs the four-wave default: MSM + Groth16 parity under it, alternated timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03r}
GM_MSM_ACCUM=idx timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "idx tests: $(tail -1 gpurun_out/${T}_tests.log)"
for rep in 1 2 3; do
  for v in def idx; do
    if [ $v = idx ]; then export GM_MSM_ACCUM=idx; else unset GM_MSM_ACCUM; fi
    for args in "--logn 20 --reps 10" "--logn 20 --reps 5 --precompute"; do
      echo -n "$v $args: "
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GM_MSM_ACCUM
cut -c1-170 gpurun_out/${T}_ab.txt
for v in def idx def idx; do
  if [ $v = idx ]; then export GM_MSM_ACCUM=idx; else unset GM_MSM_ACCUM; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json; g=json.load(open('gpurun_out/${T}_g16_$v.json'))['secondary']['groth16'][0]; print('g16 $v', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
