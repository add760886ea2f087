#!/bin/bash
# r05ai: bucket-reduction segment length (GM_MSM_SEGL) A/B on 2^24 plain-key device-input proves and the 2^20 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ai; mkdir -p $O && export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 4 16; do
    echo "== segl=$v rep $rep" >> $O/ab.txt
    if [ $v = 0 ]; then unset GM_MSM_SEGL; else export GM_MSM_SEGL=$v; fi
    timeout -k 10 300 python3 tools/g16_host_trace.py devonly >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b.json 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['kernel_avg_ms'].get('msm_bucket_reduce'))" >> $O/ab.txt
  done
done
unset GM_MSM_SEGL
grep -v "^mode" $O/ab.txt
