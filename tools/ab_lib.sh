#!/bin/bash
# Same-box A/B of the default library against gnark-icicle_amd/alt.so (GNARK_MI355X_LIB):
#   bash tools/ab_lib.sh TAG "<msm_only args>" ["<msm_only args>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for args in "$@"; do
    for lib in default alt; do
      if [ $lib = alt ]; then export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt.so; else unset GNARK_MI355X_LIB; fi
      echo -n "$lib: "
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${TAG}_ab.txt
