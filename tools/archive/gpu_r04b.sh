#!/bin/bash
# r04b: ISA issue rates incl. FP64, then the 2^24 Groth16 test with the world=8 sharded form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04b}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/isa_rate tools/microbench/isa_rate.hip || exit 1
timeout -k 10 60 /tmp/isa_rate > gpurun_out/${T}_isa_rate.txt 2>&1 || { cat gpurun_out/${T}_isa_rate.txt; exit 1; }
cat gpurun_out/${T}_isa_rate.txt
timeout -k 10 600 python -u -m pytest tests/test_configs_full.py -m gpu -x -v -s --timeout 500 --timeout-method thread -k "2p24_synthetic" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed|\[" gpurun_out/${T}_tests.log | tail -12
# plain-key 2^24 prove timeline (the default Go path)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16.json 2> gpurun_out/${T}_g16.err || { tail -30 gpurun_out/${T}_g16.err; exit 1; }
python3 -c "import json; print(json.load(open('gpurun_out/${T}_g16.json'))['secondary']['groth16'])"
python3 tools/g16_timeline.py $(ls gpurun_out/${T}_prof/prof_kernel_trace.csv gpurun_out/${T}_prof/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${T}_timeline.txt; head -40 gpurun_out/${T}_timeline.txt
rm -rf gpurun_out/${T}_prof/*/*kernel_trace.csv gpurun_out/${T}_prof/prof_kernel_trace.csv
