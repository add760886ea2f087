#!/bin/bash
# Same-box A/B of the Groth16 2^24 (precomputed) prove: computeH overlapped on
# the auxiliary stream (default) vs in order (GM_G16_OVERLAP=0), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 1 0 1 0; do
  GM_G16_OVERLAP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 \
    --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('overlap=$v', d['secondary']['groth16'][0]['prove_ms'])"
done
