#!/bin/bash
# Kernel traces of the one-frame-at-a-time bench for several --tune settings (TUNES, space-separated,
# each a comma-separated knob=value list; "-" = defaults) on CONFIG; prints the binning/sort kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for T in ${TUNES:--}; do
  O=gpurun_out/tune_${CONFIG:-3}_${T//[,=]/_}; mkdir -p $O
  A=""; [ "$T" != "-" ] && A="--tune $T"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIG:-3} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --inflight 1 --warm-ms 100 $A > $O/kt.log 2>&1 || { echo "FAILED $T"; tail -5 $O/kt.log; exit 1; }
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1
  echo "== $T  seq_fps=$(grep '^{"metric"' $O/kt.log | python3 -c 'import json,sys; print(json.load(sys.stdin)["sequential"]["value"])')"
  grep -E "k_bin_|k_radix_down|k_radix_up" $O/summary.txt | awk '{printf "   %-28s %8s\n", $1, $3}'
done
