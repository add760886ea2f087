#!/bin/bash
# r04e: uniform lane-pair Fp2 products + four-product Y3 in the G2 full adds + balanced plain windows:
# whole -m gpu suite, smoke, MSM timings, default bench, plain-key 2^24 timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=10 --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -14 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for args in "--g2 --logn 20" "--g2 --logn 20 --precompute" "--curve bls12377 --g2 --logn 22" "--curve bls12377 --logn 22" "--logn 24" "--g2 --logn 24"; do
  echo -n "$args: "; timeout -k 10 200 python tools/msm_only.py $args --reps 3 || exit 1
done 2>&1 | tee gpurun_out/${T}_msm.txt | cut -c1-200
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step']); s=d['secondary']
print(json.dumps(s['ntt'])[:200]); print(json.dumps(s['msm']))
for g in s['groth16']: print(g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'], g.get('matches_oracle'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16.json 2> gpurun_out/${T}_g16.err || { tail -30 gpurun_out/${T}_g16.err; exit 1; }
python3 tools/g16_timeline.py $(ls gpurun_out/${T}_prof/prof_kernel_trace.csv gpurun_out/${T}_prof/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${T}_timeline.txt; head -24 gpurun_out/${T}_timeline.txt
find gpurun_out/${T}_prof -name "*kernel_trace.csv" -delete
# G2 pair kernels, same box: BN254 (default = prefetch, 2 waves; PF=0; WPE=3) and BLS12-377 (3 waves vs 2 waves)
for rep in 1 2; do
  for v in def pf0 wpe3; do
    unset GM_MSM_PAIR_PF GM_MSM_PAIR_WPE
    [ $v = pf0 ] && export GM_MSM_PAIR_PF=0
    [ $v = wpe3 ] && export GM_MSM_PAIR_WPE=3
    echo -n "bn254 g2 $v: "; timeout -k 10 200 python tools/msm_only.py --g2 --logn 20 --reps 5 || exit 1
    echo -n "bn254 g2 2^24 $v: "; timeout -k 10 200 python tools/msm_only.py --g2 --logn 24 --reps 2 --precompute || exit 1
  done
  unset GM_MSM_PAIR_PF GM_MSM_PAIR_WPE
  for lib in def wpe2; do
    if [ $lib = wpe2 ]; then export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt_wpe2.so; else unset GNARK_MI355X_LIB; fi
    echo -n "bls g2 $lib: "; timeout -k 10 200 python tools/msm_only.py --curve bls12377 --g2 --logn 22 --reps 3 || exit 1
  done
  unset GNARK_MI355X_LIB
done 2>&1 | tee gpurun_out/${T}_g2_ab.txt | cut -c1-160
