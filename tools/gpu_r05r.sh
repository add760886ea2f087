#!/bin/bash
# r05r (experiment): MSM pipeline overlap vs slot-stream priority / main-stream ordering.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05r; mkdir -p $O && export TMPDIR=/tmp
for v in base prio order0 prio_order0 q8; do
  case $v in
    base) E="";; prio) E="GM_MSM_SLOT_PRIO=1";; order0) E="GM_MSM_MAIN_ORDER=0";;
    prio_order0) E="GM_MSM_SLOT_PRIO=1 GM_MSM_MAIN_ORDER=0";; q8) E="GPU_MAX_HW_QUEUES=8";;
  esac
  for rep in 1 2; do
    env $E timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep=$rep', d['value'], d['ms_per_step'], d['hip_hw_queues'])" | tee -a $O/ab.txt
  done
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o tr -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > /dev/null 2>> $O/tr.err || { tail -30 $O/tr.err; exit 1; }
  python3 tools/msm_timeline.py $(ls $O/tr_$v/*kernel_trace.csv $O/tr_$v/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/timeline_$v.txt
  find $O/tr_$v -name "*.csv" -delete
  head -1 $O/timeline_$v.txt
done
