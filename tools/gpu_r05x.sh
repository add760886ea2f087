#!/bin/bash
# r05x: kernel timeline of a 2^24 plain-key device-input Groth16 prove (where the idle gaps are).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05x; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 tools/g16_host_trace.py devonly > $O/trace.out 2> $O/trace.err || { tail -30 $O/trace.err; exit 1; }
cat $O/trace.out
python3 tools/g16_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/timeline.txt || exit 1
python3 tools/g16_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) --all > $O/timeline_all.txt || exit 1
find $O/tr -name "*.csv" -delete
head -50 $O/timeline.txt
