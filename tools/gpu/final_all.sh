#!/bin/bash
# Round-end: whole -m gpu suite + smoke (final_tests.sh), then the driver bench + rocprof cross-check (r06e.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-final}
bash tools/gpu/final_tests.sh $T && bash tools/gpu/r06e.sh $T
