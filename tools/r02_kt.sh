#!/bin/bash
# Kernel trace of the one-frame-at-a-time bench (configs in CONFIGS) + per-pass split of the
# depth-sort downsweeps (tools/pass_split.py); output under gpurun_out/kt_<config>.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
for c in ${CONFIGS:-3}; do
  O=gpurun_out/kt_$c; mkdir -p $O
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config $c --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --inflight 1 --warm-ms 200 ${BENCH_EXTRA:-} > $O/kt.log 2>&1
  rc=$?; echo "config $c kt rc=$rc"; fatal $rc kt$c; [ $rc = 0 ] || exit $rc
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1 || true
  python3 tools/pass_split.py $O k_radix_downsweep > $O/passes.txt 2>&1 || true
  head -16 $O/summary.txt; cat $O/passes.txt
done
