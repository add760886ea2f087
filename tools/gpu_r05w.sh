#!/bin/bash
# r05w (experiment): 5 MSM slots; pipeline depth 3/4/5 x reduction stream on/off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "async and not pipelined" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for d in 3 4 5; do
    for r in 0 1; do
      GM_BENCH_PIPE_DEPTH=$d GM_MSM_RED_STREAM=$r timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('depth=$d red=$r rep=$rep', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
