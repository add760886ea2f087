#!/bin/bash
# r03h: evidence for the round-3 kernels -- rocprofv3 kernel stats of the default
# bench line, SQ/GRBM VALU passes and FETCH/WRITE traffic passes over the 2^20
# G1 MSM, then the full default bench (CPU baseline + secondaries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03h}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -12 gpurun_out/${T}_rocprof_summary.txt
bash tools/gpu_pmc.sh ${T}_valu --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_pmc_valu.json gpurun_out/${T}_valu_pmc1 gpurun_out/${T}_valu_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_valu.json')); print({k: v for k, v in d.items() if 'accum' in k})"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_f -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_f.err || { tail -20 gpurun_out/${T}_f.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_w -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_w.err || { tail -20 gpurun_out/${T}_w.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_f gpurun_out/${T}_w gpurun_out/${T}_pmc_traffic.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_traffic.json')); print('accum traffic', d.get('k_msm_accum_seg'))"
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 1500 gpurun_out/${T}_bench.json; echo
