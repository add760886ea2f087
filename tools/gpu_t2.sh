mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "precomput or groth16 or msm" > gpurun_out/t2_tests.log 2>&1 || { tail -40 gpurun_out/t2_tests.log; exit 1; }
tail -3 gpurun_out/t2_tests.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline --msm-extra 1 > gpurun_out/t2_bench.json 2> gpurun_out/t2_bench.err || { tail -30 gpurun_out/t2_bench.err; exit 1; }
cat gpurun_out/t2_bench.json
