#!/bin/bash
# Round-end check of the committed tree -- the whole -m gpu suite, smoke(), the
# default bench (timed), its rocprofv3 kernel stats, and a two-rank gloo rehearsal
# of the N > 1 bench path (both ranks on the one GPU; RCCL is the driver's 8-GPU run).
#   bash tools/round_end_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-final}
bash tools/gpu_full.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -12 gpurun_out/${T}_rocprof_summary.txt
find gpurun_out/${T}_prof -name "*kernel_trace.csv" -delete
GM_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/${T}_gloo2.json 2> gpurun_out/${T}_gloo2.err || { tail -30 gpurun_out/${T}_gloo2.err; exit 1; }
head -c 800 gpurun_out/${T}_gloo2.json; echo
