#!/bin/bash
# r04d: PLONK replay (openings + domain0 FFTs), NTT tests, NTT chain A/B, plain-key 2^24 Groth16 timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04d}
timeout -k 10 900 python -u -m pytest tests/test_plonk_replay_gpu.py tests/test_ntt_gpu.py tests/test_groth16_gpu.py tests/test_pk_io_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for v in base chain; do
    if [ $v = chain ]; then export GM_NTT_CHAIN=1; else unset GM_NTT_CHAIN; fi
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22"; do
      echo -n "$v: "; timeout -k 10 120 python tools/ntt_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GM_NTT_CHAIN
cut -c1-110 gpurun_out/${T}_ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16.json 2> gpurun_out/${T}_g16.err || { tail -30 gpurun_out/${T}_g16.err; exit 1; }
python3 -c "import json; print(json.load(open('gpurun_out/${T}_g16.json'))['secondary']['groth16'])"
python3 tools/g16_timeline.py $(ls gpurun_out/${T}_prof/prof_kernel_trace.csv gpurun_out/${T}_prof/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${T}_timeline.txt; head -40 gpurun_out/${T}_timeline.txt
find gpurun_out/${T}_prof -name "*kernel_trace.csv" -delete
