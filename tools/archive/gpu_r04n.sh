#!/bin/bash
# r04n: slot streams on by default (gm_msm_async) -- MSM parity incl. the async
# tests with 8 hardware queues (real overlap), then the default bench twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04n}
timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_plonk_replay_gpu.py tests/test_icicle_replay_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q -k "async or pipelin or pending" --timeout 400 --timeout-method thread > gpurun_out/${T}_tests_q8.log 2>&1 || { tail -40 gpurun_out/${T}_tests_q8.log; exit 1; }
tail -1 gpurun_out/${T}_tests_q8.log
for rep in 1 2; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/${T}_bench$rep.json 2> gpurun_out/${T}_bench$rep.err || { tail -20 gpurun_out/${T}_bench$rep.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench$rep.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'], d['roofline']['frac'], d['roofline']['int_alu']['frac'])
s=d['secondary']; print(json.dumps(s['ntt'])[:300]); print(json.dumps(s['msm']))
for g in s['groth16']: print(g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
