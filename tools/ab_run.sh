#!/bin/bash
# Same-box A/B runner (the pattern behind the profiles/r0*_ab.txt files): runs COMMAND once per
# environment variant, alternating variants in fresh processes for REPS rounds, each run under its own
# time limit, and appends "variant | output" lines to OUT.  Stops at the first failing run.
#   bash tools/ab_run.sh OUT REPS "GM_X=0" "GM_X=1" -- python3 tools/msm_only.py --logn 20 --reps 5
#   bash tools/ab_run.sh gpurun_out/ab.txt 2 "" "GM_G16_H_INCREMENTAL=0" -- python3 tools/g16_host_trace.py devonly
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; REPS=$2; shift 2
VARIANTS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARIANTS+=("$1"); shift; done
[ "$1" = "--" ] || { echo "usage: ab_run.sh OUT REPS VARIANT... -- COMMAND..." >&2; exit 2; }
shift
mkdir -p "$(dirname "$OUT")" && export TMPDIR=/tmp
for rep in $(seq 1 "$REPS"); do
  for v in "${VARIANTS[@]}"; do
    res=$(env $v timeout -k 10 "${AB_TIMEOUT:-300}" "$@" 2>> "$OUT.err") || { echo "failed: [$v] $*" >&2; tail -20 "$OUT.err" >&2; exit 1; }
    echo "$res" | sed "s%^%[${v:-default}] rep $rep | %" | tee -a "$OUT"
  done
done
