#!/bin/bash
# r04ab: the default bench line (no CPU baselines / secondary) twice, new defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/r04ab_$i.json 2> gpurun_out/r04ab_$i.err || { tail -20 gpurun_out/r04ab_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r04ab_$i.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['steps'], r['avg_launch_ms'], r['frac'], r['int_alu']['frac'], r['isolated'])"
done
