#!/bin/bash
# r03n: round-3 final check -- full -m gpu suite, smoke, default bench under
# rocprofv3 --kernel-trace --stats, NTT 2^24 VALU / traffic counter passes,
# then the full default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03n}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -6 gpurun_out/${T}_rocprof_summary.txt
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_ntt_pmc_valu.json gpurun_out/${T}_ntt_pmc1 gpurun_out/${T}_ntt_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_ntt_pmc_valu.json')); print({k: v for k, v in d.items() if 'ntt' in k})"
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 900 gpurun_out/${T}_bench.json; echo
