#!/bin/bash
# r05g: MSM parity with the v4 key / value groups, then a same-box A/B of
# GM_MSM_ACC_V4=1 (default) vs 0: bench MSM line x3 each, FETCH_SIZE of the
# accumulation, Groth16 2^24 x2 each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_msm_gpu.py tests/test_golden_gpu.py tests/test_groth16_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do
  for v in 1 0; do
    GM_MSM_ACC_V4=$v timeout -k 10 200 python -u bench.py --no-secondary --no-cpu-baseline --steps 30 > $O/msm_v$v.$i.json 2>> $O/err.txt || { tail -30 $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('$O/msm_v$v.$i.json')); print('v4=$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['isolated']['avg_launch_ms'])"
  done
done
for v in 1 0; do
  GM_MSM_ACC_V4=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$v -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> $O/f$v.err || { tail -20 $O/f$v.err; exit 1; }
  python3 -c "
import csv, glob
v = [float(r['Counter_Value']) for f in glob.glob('$O/f$v/**/*counter_collection*.csv', recursive=True) for r in csv.DictReader(open(f)) if 'accum' in r['Kernel_Name']]
print('v4=$v accumulation FETCH_SIZE per launch: %.3f GB (raw tally, %d launches)' % (sum(v) / len(v) * 1024 / 1e9, len(v)))"
done
find $O -name "*.csv" -size +5M -delete
for i in 1 2; do
  for v in 1 0; do
    GM_MSM_ACC_V4=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --msm-extra 0 --g16-logn 24 --g16-plain 24 > $O/g16_v$v.$i.json 2>> $O/err.txt || { tail -30 $O/err.txt; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/g16_v$v.$i.json'))
print('v4=$v', [(g['pk'], g['prove_ms_device_inputs'], g['prove_ms_host_inputs']) for g in d['secondary']['groth16']])"
  done
done
