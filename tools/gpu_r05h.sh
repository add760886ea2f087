#!/bin/bash
# r05h: parity of the v4 key / value groups in every accumulation kernel (G1 chain,
# BLS12-377 G1 prefetching, G2 lane pairs), then same-box A/B GM_MSM_ACC_V4=1 vs 0:
# the bench's extra MSM lines (BN254 G2 2^20, BLS12-377 G1 / G2 2^22) and Groth16 2^24.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05h; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_golden_gpu.py tests/test_configs_full.py -k "not 2p24_synthetic" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  for v in 1 0; do
    GM_MSM_ACC_V4=$v timeout -k 10 400 python -u bench.py --steps 10 --no-cpu-baseline --g16-logn 24 --g16-plain 24 > $O/b_v$v.$i.json 2>> $O/err.txt || { tail -30 $O/err.txt; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_v$v.$i.json')); s=d['secondary']
print('v4=$v', d['value'], {k: v['ms'] for k, v in s['msm'].items()}, [(g['pk'], g['prove_ms_device_inputs'], g['prove_ms_host_inputs']) for g in s['groth16']])"
  done
done
