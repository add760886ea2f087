#!/bin/bash
# r04v: a / b / c of host-input proves in their own allocation (gm_ctx::in_abc):
# parity, fresh-process 2^24 host-input proves, and the full default bench's
# Groth16 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04v}
timeout -k 10 900 python -u -m pytest tests/test_groth16_gpu.py tests/test_configs_full.py tests/test_pk_io_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python3 -u tools/g16_host_trace.py fresh 2>&1 | grep -E "mode|prove" | tee gpurun_out/${T}_fresh.txt || exit 1
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('msm', d['value'], d['ms_per_step'])
for g in d['secondary']['groth16']: print('g16', g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
