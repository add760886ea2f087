#!/bin/bash
# r05e: second-stream / trim tests, then a same-box A/B of the accumulation-only
# mad-chain kernel (GM_MSM_ACC_CHAIN=1): bench MSM line x3 each, Groth16 2^24 x2 each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05e; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_groth16_gpu.py -k "second_msm_stream or trim" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2 3; do
  for v in 0 1; do
    GM_MSM_ACC_CHAIN=$v timeout -k 10 200 python -u bench.py --no-secondary --no-cpu-baseline --steps 30 > $O/msm_ch$v.$i.json 2>> $O/err.txt || { tail -30 $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('$O/msm_ch$v.$i.json')); print('chain=$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['isolated']['avg_launch_ms'])"
  done
done
for i in 1 2; do
  for v in 0 1; do
    GM_MSM_ACC_CHAIN=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --msm-extra 0 --g16-logn 24 --g16-plain 24 > $O/g16_ch$v.$i.json 2>> $O/err.txt || { tail -30 $O/err.txt; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/g16_ch$v.$i.json'))
print('chain=$v', [(g['pk'], g['prove_ms_device_inputs'], g['prove_ms_host_inputs']) for g in d['secondary']['groth16']])"
  done
done
