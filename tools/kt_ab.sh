#!/bin/bash
# Kernel trace of the one-frame-at-a-time bench for two knob settings (A/B per kernel):
# TUNES="19=0 19=1" CONFIG=2; summaries under gpurun_out/kt_ab_<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
for t in ${TUNES:-19=0 19=1}; do
  tag=$(echo "$t" | tr '=,' '__')
  O=gpurun_out/kt_ab_$tag; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIG:-2} --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --inflight 1 --warm-ms 200 --tune "$t" > $O/kt.log 2>&1
  rc=$?; echo "tune $t kt rc=$rc"; fatal $rc kt; [ $rc = 0 ] || exit $rc
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1 || true
  echo "== $t"; head -16 $O/summary.txt
done
