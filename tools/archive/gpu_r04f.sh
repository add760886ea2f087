#!/bin/bash
# r04f: G1 Y3 as one unsigned reduction (R W + (5p - Y1) PPP) and BLS12-377 G2 pairs at two waves:
# MSM / Groth16 parity, same-box A/B vs the previous commit (alt_g1old.so), H2D rates, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04f}
timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2 3; do
  for lib in new old; do
    if [ $lib = old ]; then export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt_g1old.so; else unset GNARK_MI355X_LIB; fi
    for args in "--logn 20" "--logn 20 --precompute" "--logn 24 --precompute" "--curve bls12377 --logn 22"; do
      echo -n "$lib $args: "; timeout -k 10 200 python tools/msm_only.py $args --reps 5 || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_ab.txt | cut -c1-170
unset GNARK_MI355X_LIB
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/h2d tools/microbench/h2d.hip -lpthread && timeout -k 10 120 /tmp/h2d > gpurun_out/${T}_h2d.txt 2>&1; cat gpurun_out/${T}_h2d.txt
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_ms']); s=d['secondary']
print(json.dumps(s['msm']))
for g in s['groth16']: print(g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
# host-input Groth16 2^24 (precomputed): staged pinned ring vs pageable hipMemcpyAsync, same box
for v in staged pageable staged pageable; do
  if [ $v = pageable ]; then export GM_H2D=pageable; else unset GM_H2D; fi
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain "" --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_h2d_$v.json 2> gpurun_out/${T}_h2d_$v.err || { tail -20 gpurun_out/${T}_h2d_$v.err; exit 1; }
  python3 -c "
import json; g=json.load(open('gpurun_out/${T}_h2d_$v.json'))['secondary']['groth16'][0]; print('$v', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
unset GM_H2D
