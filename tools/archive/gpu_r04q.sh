#!/bin/bash
# r04q: which earlier part of the full bench slows the later 2^24 plain host-input
# prove (200 ms vs 167 in a reduced run)?  Bisect the sequence, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04q}
i=0
for args in "--msm-extra 0 --ntt-logn 20 --g16-logn 24" "--msm-extra 0 --ntt-logn 20 --g16-logn 20,24" "--msm-extra 1 --ntt-logn 20 --g16-logn 24" "--msm-extra 0 --ntt-logn 24 --g16-logn 24"; do
  i=$((i+1))
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --g16-no-precomputed $args > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err || { tail -20 gpurun_out/${T}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json'))
for g in d['secondary']['groth16']: print('$args |', g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])" | tee -a gpurun_out/${T}_ab.txt
done
