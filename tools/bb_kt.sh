#!/bin/bash
# Kernel trace of tools/bb_probe.py (config 3, a steady 0.25-deg orbit, one frame at a time)
# for each BUCKETS value (knob 28): the per-kernel means without the bench's camera jumps.
# KT_TAG names an A/B variant (its env set by the caller) in the output directory.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for b in ${BUCKETS_LIST:-0 1}; do
  O=gpurun_out/bbkt_$b${KT_TAG:-}; mkdir -p $O
  BUCKETS=$b FRAMES=${FRAMES:-120} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/bb_probe.py > $O/kt.log 2>&1
  rc=$?; echo "buckets $b rc=$rc"; [ $rc = 0 ] || exit $rc
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; echo "== 28=$b ${KT_TAG:-}"; head -22 $O/summary.txt
  find $O -name "*kernel_trace.csv" -delete
done
