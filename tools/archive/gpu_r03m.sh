#!/bin/bash
# r03m: NTT twiddles through the cache (GM_NTT_SWG=1: four blocks per CU) with the
# interleaved butterflies -- parity, then alternated 2^24 timings vs the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03m}
GM_NTT_SWG=1 timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "swg tests: $(tail -1 gpurun_out/${T}_tests.log)"
for rep in 1 2 3; do
  for v in 0 1; do
    for args in "--logn 24 --reps 4" "--logn 24 --reps 4 --coset"; do
      echo -n "swg=$v $args: "
      GM_NTT_SWG=$v timeout -k 10 200 python tools/ntt_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
cut -c1-130 gpurun_out/${T}_ab.txt
