#!/bin/bash
# r04p: the full default bench (as the driver runs it, minus the CPU baselines) with
# GPU_MAX_HW_QUEUES 4 vs 8, same box -- r04n's 2^24 plain host-input prove took 199 ms
# in the full sequence against 167 in the reduced one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04p}
for q in 8 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/${T}_q$q.json 2> gpurun_out/${T}_q$q.err || { tail -20 gpurun_out/${T}_q$q.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_q$q.json')); print('q=$q msm', d['value'], d['ms_per_step'])
for g in d['secondary']['groth16']: print('q=$q g16', g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'], g['best_ms'])" | tee -a gpurun_out/${T}_ab.txt
done
