#!/bin/bash
# r05i: copy + kernel trace of 2^24 host-input proves (plain key), the kernel stats of the
# default bench line, then the counters of the final kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05i; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 tools/g16_host_trace.py > $O/trace.out 2> $O/trace.err || { tail -30 $O/trace.err; exit 1; }
cat $O/trace.out
python3 tools/g16_copy_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) $(ls $O/tr/*memory_copy_trace.csv $O/tr/*/*memory_copy_trace.csv 2>/dev/null | head -1) > $O/host_prove_timeline.txt || exit 1
head -40 $O/host_prove_timeline.txt
find $O -name "*.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05j_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/r05j_profbench.json 2> gpurun_out/r05j_prof.err || { tail -30 gpurun_out/r05j_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/r05j_prof/*kernel_stats.csv gpurun_out/r05j_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/r05j_rocprof_summary.txt && head -8 gpurun_out/r05j_rocprof_summary.txt
find gpurun_out/r05j_prof -name "*kernel_trace.csv" -delete
# counters of the final kernels (r05j): VALU passes over the 2^20 G1 MSM, the 2^20 G2
# MSM and the 2^24 NTT; FETCH / WRITE over the G1 MSM
T=r05j
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
