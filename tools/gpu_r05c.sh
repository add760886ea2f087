#!/bin/bash
# r05c: staged-input tests, then the default bench (all secondaries) timed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05c; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pk_io_gpu.py > $O/pk_io_tests.txt 2>&1 || { tail -30 $O/pk_io_tests.txt; exit 1; }
tail -3 $O/pk_io_tests.txt
start=$SECONDS
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "default bench wall: $((SECONDS - start)) s"
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])
for g in d['secondary']['groth16']: print({k: v for k, v in g.items() if k not in ('roofline', 'pk_dump')})
print(d['secondary']['ntt']['ms_per_transform'])"
