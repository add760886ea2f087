#!/bin/bash
# r04ae: accumulation slice length (GM_MSM_SLICE) with three MSMs in flight: parity at
# 32, the 2^20 bench line for 16..64, and the Groth16 2^24 proves at 32 vs 64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04ae}
GM_MSM_SLICE=32 timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for k in 64 48 32 24 16; do
    GM_MSM_SLICE=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}.json')); print('K=$k', d['value'], d['ms_per_step'], d['roofline']['isolated']['avg_launch_ms'])" | tee -a gpurun_out/${T}_sweep.txt
  done
done
for k in 32 64; do
  GM_MSM_SLICE=$k timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --g16-logn 24 --g16-plain 24 --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16_$k.json 2> gpurun_out/${T}_g16_$k.err || { tail -20 gpurun_out/${T}_g16_$k.err; exit 1; }
  python3 -c "
import json
for g in json.load(open('gpurun_out/${T}_g16_$k.json'))['secondary']['groth16']: print('K=$k g16 2^%d' % g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'])" | tee -a gpurun_out/${T}_sweep.txt
done
