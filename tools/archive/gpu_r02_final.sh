#!/bin/bash
# Round-2 verification pass on one MI355X: full -m gpu suite, smoke, default bench,
# rocprofv3 kernel stats of the primary bench, FETCH/WRITE traffic, VALU counters
# (2^20) and the accumulation's gather traffic at 2^24 (plain and precomputed).
#   bash tools/gpu_r02_final.sh TAG [notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02f}
if [ "${2:-}" != notests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=20 --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
  tail -3 gpurun_out/${T}_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 400 gpurun_out/${T}_bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmcf -o pmc -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > /dev/null 2> gpurun_out/${T}_pmcf.err || { tail -20 gpurun_out/${T}_pmcf.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmcw -o pmc -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > /dev/null 2> gpurun_out/${T}_pmcw.err || { tail -20 gpurun_out/${T}_pmcw.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_pmcf gpurun_out/${T}_pmcw gpurun_out/${T}_pmc_traffic.json > /dev/null
bash tools/gpu_pmc.sh ${T}_valu --reps 3 > /dev/null || exit 1
for mode in "" "--precompute"; do
  tag=${T}_g24$( [ -n "$mode" ] && echo pre || echo plain )
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag} -o pmc -- python3 tools/msm_only.py --logn 24 --reps 1 $mode > gpurun_out/${tag}.out 2>&1 || { tail -5 gpurun_out/${tag}.out; exit 1; }
done
echo done
