#!/bin/bash
# r05d: staged wires + resident R1CS tests, then the Groth16 secondaries of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05d; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_r1cs_gpu.py tests/test_pk_io_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python -u bench.py --steps 10 --msm-extra 0 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
for g in d['secondary']['groth16']: print({k: v for k, v in g.items() if k.startswith('prove_ms') or 'match' in k})"
