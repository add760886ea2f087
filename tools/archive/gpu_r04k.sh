#!/bin/bash
# r04k: Groth16 slot-1 MSMs (B, B2, Z) on a second stream (GM_G16_MSM_STREAMS=1):
# proof parity with it on, then same-box A/B of the 2^24 prove (plain and
# precomputed keys) and a kernel-trace timeline of one 2^24 plain prove each way.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04k}
GM_G16_MSM_STREAMS=1 timeout -k 10 900 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_configs_full.py tests/test_icicle_replay_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in 0 1 0 1; do
  GM_G16_MSM_STREAMS=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json
for g in json.load(open('gpurun_out/${T}_g16_$v.json'))['secondary']['groth16']: print('streams=$v g16 2^%d' % g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])" | tee -a gpurun_out/${T}_g16_ab.txt
done
for v in 0 1; do
  GM_G16_MSM_STREAMS=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt$v -o kt -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --msm-extra 0 --ntt-logn 20 > /dev/null 2> gpurun_out/${T}_kt$v.err || { tail -20 gpurun_out/${T}_kt$v.err; exit 1; }
  F=$(ls gpurun_out/${T}_kt$v/*kernel_trace.csv gpurun_out/${T}_kt$v/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/g16_timeline.py $F > gpurun_out/${T}_timeline_$v.txt && head -14 gpurun_out/${T}_timeline_$v.txt
  find gpurun_out/${T}_kt$v -name "*.csv" -size +5M -delete
done
