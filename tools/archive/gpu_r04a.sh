#!/bin/bash
# r04a: baseline of the round-4 box: smoke, then the default bench (now incl. the plain-key 2^24 prove).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04a}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
start=$SECONDS
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
echo "default bench wall: $((SECONDS - start)) s"
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step']); s=d['secondary']
print(json.dumps(s['ntt'])[:300]); print(json.dumps(s['msm']))
for g in s['groth16']: print(g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
