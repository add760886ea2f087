#!/bin/bash
# r03g: NTT launch-shape variants (GM_NTT_TPB=512 one butterfly per thread and
# stage, GM_NTT_SWG=1 twiddles through the cache) -- parity tests under each,
# then 2^24 timings alternated; Groth16 2^24 prove with the 3-wave prefetching
# G1 accumulation (GM_MSM_ACCUM=prefetch) vs the 4-wave default, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03g}
for v in "256 0" "512 0" "256 1" "512 1"; do
  set -- $v
  GM_NTT_TPB=$1 GM_NTT_SWG=$2 timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_ntt_tests_$1_$2.log 2>&1 || { tail -30 gpurun_out/${T}_ntt_tests_$1_$2.log; exit 1; }
  echo "tpb=$1 swg=$2 $(tail -1 gpurun_out/${T}_ntt_tests_$1_$2.log)"
done
for rep in 1 2; do
  for v in "256 0" "512 0" "256 1" "512 1"; do
    set -- $v
    for args in "--logn 24 --reps 4" "--logn 24 --reps 4 --coset"; do
      echo -n "tpb=$1 swg=$2 $args: "
      GM_NTT_TPB=$1 GM_NTT_SWG=$2 timeout -k 10 200 python tools/ntt_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ntt_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ntt_ab.txt; exit 1; }
cat gpurun_out/${T}_ntt_ab.txt | cut -c1-130
for v in default prefetch default prefetch; do
  unset GM_MSM_ACCUM
  [ $v = prefetch ] && export GM_MSM_ACCUM=prefetch
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g16_$v.json')); g=d['secondary']['groth16'][0]; print('$v', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
