#!/bin/bash
# SQ / GRBM counter passes over tools/msm_only.py (one rocprofv3 --pmc run per
# pass, counters filtered against `rocprofv3 -L`).
#   bash tools/gpu_pmc.sh TAG [msm_only.py args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; shift
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/${T}_counters.txt; }
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MUL_U32 SQ_INST_CYCLES_SALU GRBM_COUNT"
k=0
for P in "$P1" "$P2"; do
  k=$((k+1)); L=""; n=0
  for c in $P; do
    if have $c; then
      case $c in SQ_*) n=$((n+1)); [ $n -gt 8 ] && continue;; esac
      L="$L $c"
    fi
  done
  echo "pass $k:$L"
  timeout -s KILL 90 rocprofv3 --pmc $L --output-format csv -d gpurun_out/${T}_pmc$k -o pmc -- python3 ${PROG:-tools/msm_only.py} "$@" > gpurun_out/${T}_pmc$k.out 2>&1 || { tail -5 gpurun_out/${T}_pmc$k.out; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${T}_pmc1 gpurun_out/${T}_pmc2 > gpurun_out/${T}_pmc_summary.txt && cat gpurun_out/${T}_pmc_summary.txt
