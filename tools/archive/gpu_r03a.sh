#!/bin/bash
# r03a: MSM / pk-io / Groth16 GPU tests after the narrow-window precompute
# layout, BLS12-377 GLV and the readback-buffer change; MSM timings; 2^24
# Groth16 kernel timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03a}
timeout -k 10 700 python -u -m pytest tests/test_msm_gpu.py tests/test_pk_io_gpu.py tests/test_groth16_gpu.py tests/test_plonk_replay_gpu.py tests/test_r1cs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for args in "--logn 20" "--logn 20 --precompute" "--logn 24 --precompute --reps 3" "--g2 --logn 20" "--g2 --logn 24 --precompute --reps 2" "--curve bls12377 --logn 22 --reps 3" "--curve bls12377 --g2 --logn 22 --reps 2"; do
  timeout -k 10 300 python3 tools/msm_only.py $args >> gpurun_out/${T}_msm.txt 2>&1 || { tail -5 gpurun_out/${T}_msm.txt; exit 1; }
done
cat gpurun_out/${T}_msm.txt
bash tools/gpu_g16.sh ${T}_g16 notests
