#!/bin/bash
# r04o: GPU_MAX_HW_QUEUES 4 vs 8 (bench.py sets 8 unless the environment says
# otherwise), same box: MSM headline and the Groth16 2^24 proves (plain host inputs
# regressed 166 -> 199 ms in r04n).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04o}
for rep in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python3 bench.py --no-cpu-baseline --msm-extra 0 --ntt-logn 20 --g16-logn 24 > gpurun_out/${T}_q$q.json 2> gpurun_out/${T}_q$q.err || { tail -20 gpurun_out/${T}_q$q.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_q$q.json')); print('q=$q msm', d['value'], d['ms_per_step'])
for g in d['secondary']['groth16']: print('q=$q g16', g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])" | tee -a gpurun_out/${T}_ab.txt
  done
done
