#!/bin/bash
# r03o: bench with the sharded steps pipelined -- N=1 line, then the N>1 code
# path rehearsed on the one-GPU box (2 and 4 ranks on cuda:0 over gloo; RCCL
# needs one GPU per rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03o}
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_n1.json 2> gpurun_out/${T}_n1.err || { tail -30 gpurun_out/${T}_n1.err; exit 1; }
head -c 300 gpurun_out/${T}_n1.json; echo
for N in 2 4; do
  GM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/${T}_n$N.json 2> gpurun_out/${T}_n$N.err || { tail -30 gpurun_out/${T}_n$N.err; exit 1; }
  head -c 300 gpurun_out/${T}_n$N.json; echo
done
