#!/bin/bash
# r04g: round-4 evidence -- rocprofv3 kernel stats of the default bench line, VALU counter passes
# over the 2^20 G1 MSM, the 2^20 G2 MSM and the 2^24 NTT, FETCH / WRITE traffic passes over the G1 MSM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04g}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -12 gpurun_out/${T}_rocprof_summary.txt
find gpurun_out/${T}_prof -name "*kernel_trace.csv" -delete
bash tools/gpu_pmc.sh ${T}_valu --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_pmc_valu.json gpurun_out/${T}_valu_pmc1 gpurun_out/${T}_valu_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_valu.json')); print({k: v for k, v in d.items() if 'accum' in k})"
bash tools/gpu_pmc.sh ${T}_g2valu --g2 --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_g2_pmc_valu.json gpurun_out/${T}_g2valu_pmc1 gpurun_out/${T}_g2valu_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_g2_pmc_valu.json')); print({k: v for k, v in d.items() if 'pair' in k})"
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_ntt_pmc_valu.json gpurun_out/${T}_ntt_pmc1 gpurun_out/${T}_ntt_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_ntt_pmc_valu.json')); print({k: v for k, v in d.items() if 'ntt' in k})"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_f -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_f.err || { tail -20 gpurun_out/${T}_f.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_w -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_w.err || { tail -20 gpurun_out/${T}_w.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_f gpurun_out/${T}_w gpurun_out/${T}_pmc_traffic.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_traffic.json')); print('accum traffic', d.get('k_msm_accum_seg'))"
find gpurun_out/${T}_* -name "*.csv" -size +5M -delete
