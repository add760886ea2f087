#!/bin/bash
# r06s: h first (GM_G16_H_FIRST=1 build): computeH queued at the start of a device-input prove beside the wire
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06s_*.txt was measured)
# plan's sort, the MSMs wait for h, and Z's digits / sort follow computeH on the auxiliary stream (third slot) beside
# A's accumulation -- vs computeH after the wire plan beside the accumulations, Z planned after K (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_hf.so"
env $ALT timeout -k 10 600 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s_tests.log 2>&1 || { tail -30 gpurun_out/r06s_tests.log; exit 1; }
tail -1 gpurun_out/r06s_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06s_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06s_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06s_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 20 --reps 5 || exit 1
env $ALT timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06s_kt -o kt -- python3 tools/g16_only.py --logn 24 --reps 1 > gpurun_out/r06s_kt.out 2>&1 || { tail -5 gpurun_out/r06s_kt.out; exit 1; }
TR=$(find gpurun_out/r06s_kt -name "*kernel_trace.csv" | head -1)
python3 tools/g16_exposed.py "$TR" | tee gpurun_out/r06s_exposed.txt
gzip -f "$TR"
