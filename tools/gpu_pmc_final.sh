#!/bin/bash
# Counter passes of the final kernels for the bench line's roofline fields: VALU passes over the 2^20 G1 MSM,
# the 2^20 G2 MSM and the 2^24 NTT; FETCH_SIZE / WRITE_SIZE passes over the G1 MSM (each pass a run of its own).
#   bash tools/gpu_pmc_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-final}
export TMPDIR=/tmp
bash tools/gpu_pmc.sh ${T}_valu --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_pmc_valu.json gpurun_out/${T}_valu_pmc1 gpurun_out/${T}_valu_pmc2 > /dev/null || exit 1
bash tools/gpu_pmc.sh ${T}_g2valu --g2 --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_g2_pmc_valu.json gpurun_out/${T}_g2valu_pmc1 gpurun_out/${T}_g2valu_pmc2 > /dev/null || exit 1
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_ntt_pmc_valu.json gpurun_out/${T}_ntt_pmc1 gpurun_out/${T}_ntt_pmc2 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_f -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_f.err || { tail -20 gpurun_out/${T}_f.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_w -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_w.err || { tail -20 gpurun_out/${T}_w.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_f gpurun_out/${T}_w gpurun_out/${T}_pmc_traffic.json > /dev/null || exit 1
python3 -c "
import json
for f in ('${T}_pmc_valu', '${T}_g2_pmc_valu', '${T}_ntt_pmc_valu'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, {k: v for k, v in d.items() if 'accum' in k or 'ntt' in k})
d = json.load(open('gpurun_out/${T}_pmc_traffic.json')); print('fetch KiB', {k: v for k, v in d['_meta']['fetch_kib'].items() if 'accum' in k})"
find gpurun_out/${T}_* -name "*.csv" -size +5M -delete
