#!/bin/bash
# r03w: the driver's N>1 invocation rehearsed on one GPU (2 gloo ranks sharing
# cuda:0; gm_multi maps its devices modulo the visible GPUs) with every default
# secondary on: sharded Groth16 2^24 and the single-process gm_multi prove.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03w}
start=$(date +%s)
GM_BENCH_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/${T}_n2.json 2> gpurun_out/${T}_n2.err || { tail -40 gpurun_out/${T}_n2.err; exit 1; }
echo "elapsed $(( $(date +%s) - start )) s"
grep -o '{"metric.*' gpurun_out/${T}_n2.json | head -c 2500; echo
