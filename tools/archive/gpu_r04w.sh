#!/bin/bash
# r04w: host-input a/b/c through the context's pinned ring (GM_G16_H2D_PINNED, default
# on) vs pageable copies: parity, fresh-process and device-first 2^24 proves, and the
# reduced bench's 2^24 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04w}
timeout -k 10 900 python -u -m pytest tests/test_groth16_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for p in 1 0; do
  for m in fresh device; do
    echo "GM_G16_H2D_PINNED=$p" | tee -a gpurun_out/${T}.txt
    GM_G16_H2D_PINNED=$p timeout -k 10 300 python3 -u tools/g16_host_trace.py $m 2>&1 | grep -E "mode|prove" | tee -a gpurun_out/${T}.txt || exit 1
  done
done
for p in 1 0; do
  GM_G16_H2D_PINNED=$p timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16_$p.json 2> gpurun_out/${T}_g16_$p.err || { tail -20 gpurun_out/${T}_g16_$p.err; exit 1; }
  python3 -c "
import json
for g in json.load(open('gpurun_out/${T}_g16_$p.json'))['secondary']['groth16']: print('pinned=$p g16 2^%d' % g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])" | tee -a gpurun_out/${T}.txt
done
