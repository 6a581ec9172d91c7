#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the bench for configs 2 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2 gpurun_out/prof3
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
for c in ${CONFIGS:-2 3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$c/kt -o kt --output-format csv -- python3 bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --warm-ms 300 > gpurun_out/prof$c/kt.log 2>&1
  rc=$?; echo "config $c kt rc=$rc"; fatal $rc kt$c; [ $rc = 0 ] || exit $rc
  python3 tools/summarize_prof.py gpurun_out/prof$c > gpurun_out/prof$c/summary.txt 2>&1 || true
done
