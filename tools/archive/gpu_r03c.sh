#!/bin/bash
# r03c: R1CS / Groth16 / MSM GPU tests after dropping the skipped-entry branch
# and queueing the R1CS evaluation at prove start; BLS12-377 MSM timings;
# Groth16 2^24 timeline; NTT 2^24 counter passes (VALU, HBM traffic); the
# default bench under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03c}
timeout -k 10 700 python -u -m pytest tests/test_r1cs_gpu.py tests/test_groth16_gpu.py tests/test_msm_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for args in "--curve bls12377 --logn 22 --reps 3" "--curve bls12377 --g2 --logn 22 --reps 2"; do
  timeout -k 10 300 python3 tools/msm_only.py $args >> gpurun_out/${T}_msm.txt 2>&1 || { tail -5 gpurun_out/${T}_msm.txt; exit 1; }
done
cat gpurun_out/${T}_msm.txt
bash tools/gpu_g16.sh ${T}_g16 notests || exit 1
timeout -k 10 120 python3 tools/ntt_only.py --logn 24 > gpurun_out/${T}_ntt.txt 2>&1 && timeout -k 10 120 python3 tools/ntt_only.py --logn 24 --coset >> gpurun_out/${T}_ntt.txt 2>&1 || { tail -5 gpurun_out/${T}_ntt.txt; exit 1; }
cat gpurun_out/${T}_ntt.txt
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_nttf -o pmc -- python3 tools/ntt_only.py --logn 24 --reps 2 > /dev/null 2> gpurun_out/${T}_nttf.err || { tail -20 gpurun_out/${T}_nttf.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_nttw -o pmc -- python3 tools/ntt_only.py --logn 24 --reps 2 > /dev/null 2> gpurun_out/${T}_nttw.err || { tail -20 gpurun_out/${T}_nttw.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_nttf gpurun_out/${T}_nttw gpurun_out/${T}_ntt_traffic.json > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -c 400 gpurun_out/${T}_profbench.json; echo
echo done
