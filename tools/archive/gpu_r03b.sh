#!/bin/bash
# r03b: full -m gpu suite, smoke, default bench, msm timings, Groth16 2^24
# timelines with computeH queued after / with the shared wire plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for args in "--curve bls12377 --logn 22 --reps 3" "--curve bls12377 --g2 --logn 22 --reps 2" "--g2 --logn 20"; do
  timeout -k 10 300 python3 tools/msm_only.py $args >> gpurun_out/${T}_msm.txt 2>&1 || { tail -5 gpurun_out/${T}_msm.txt; exit 1; }
done
cat gpurun_out/${T}_msm.txt
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 300 gpurun_out/${T}_bench.json; echo
bash tools/gpu_g16.sh ${T}_g16 notests || exit 1
GM_G16_H_AFTER_PLAN=0 bash tools/gpu_g16.sh ${T}_g16now notests || exit 1
