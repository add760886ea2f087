#!/bin/bash
# Same-box A/B runner (the pattern behind the profiles/r0*_ab.txt files): runs COMMAND once per
# environment variant, alternating variants in fresh processes for REPS rounds, each run under its own
# time limit, and appends "variant | output" lines to OUT.  Stops at the first failing run.
#   bash tools/ab_run.sh OUT REPS "" "GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_alt.so" -- python3 tools/msm_only.py
# (the variant is an alternative build of the library, or any environment the command reads)
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
