#!/bin/bash
# Kernel trace of the frames-in-flight bench (config CONFIG, default 4 lanes) and the gap
# analysis between consecutive blends (tools/blend_gaps.py, tools/inflight_gaps.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/ifkt_${CONFIG:-2}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIG:-2} --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --warm-ms 200 ${BENCH_EXTRA:-} > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
python3 tools/blend_gaps.py $O/kt/kt_kernel_trace.csv > $O/blend_gaps.txt 2>&1
python3 tools/inflight_gaps.py $O/kt/kt_kernel_trace.csv > $O/inflight_gaps.txt 2>&1
cat $O/blend_gaps.txt; head -40 $O/inflight_gaps.txt
