#!/bin/bash
# Full GPU pass + N=2 rehearsal of the multi-rank bench path (gloo, one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-t6}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
GM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --g16-sharded-logn 22 > gpurun_out/${TAG}_n2.json 2> gpurun_out/${TAG}_n2.err || { tail -30 gpurun_out/${TAG}_n2.err; exit 1; }
cat gpurun_out/${TAG}_n2.json
