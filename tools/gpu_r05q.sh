#!/bin/bash
# r05q: staged put_range filled by four threads: pk-io / Groth16 tests, then the 2^24 plain-key
# Groth16 scopes of the bench (staged wires-after-solve scope) with GM_G16_H2D_THREADS=1 vs default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pk_io_gpu.py tests/test_groth16_gpu.py tests/test_r1cs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 4; do
  GM_G16_H2D_THREADS=$v timeout -k 10 600 python3 bench.py --no-cpu-baseline --msm-extra 0 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --steps 5 > $O/b_$v.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1])
g=d['secondary']['groth16'][0]
print('threads=$v', {k: v for k, v in g.items() if k.startswith('prove_ms')})" | tee -a $O/ab.txt
done
