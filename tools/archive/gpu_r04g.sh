#!/bin/bash
# r04g: growing-bound DIF rounds (GM_NTT_GROW) parity + same-box A/B, the FP64-limb Montgomery
# microbench, then round-4 evidence -- rocprofv3 kernel stats of the default bench line, VALU counter
# passes over the 2^20 G1 MSM, the 2^20 G2 MSM and the 2^24 NTT, FETCH / WRITE traffic over the G1 MSM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04g}
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_configs_full.py tests/test_groth16_gpu.py tests/test_icicle_replay_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2 3; do
  for g in 1 0; do
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22" "--logn 20"; do
      echo -n "grow=$g $args: "; GM_NTT_GROW=$g timeout -k 10 120 python3 tools/ntt_only.py $args || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_ntt_grow_ab.txt | cut -c1-150
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -o /tmp/fp64mont tools/microbench/fp64mont.hip && timeout -k 10 60 /tmp/fp64mont /tmp/fp64mont_dump.txt > gpurun_out/${T}_fp64mont.txt 2>&1 && python3 tools/microbench/fp64mont_check.py /tmp/fp64mont_dump.txt >> gpurun_out/${T}_fp64mont.txt; cat gpurun_out/${T}_fp64mont.txt
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
