#!/bin/bash
# Interleaved end-to-end A/B of knob 28 at config 3 (5M): the LSD passes (1 before the big
# buckets were the default above 2M, 0 after) against the big buckets (4 / 1), fixed camera and
# a 0.25-deg orbit, ROUNDS rounds, one process per run.  Prints in-flight and one-at-a-time frames/s.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abc3
for i in $(seq 1 ${ROUNDS:-2}); do
  for t in ${KNOBS:-0 1}; do
    for o in 0 0.25; do
      L=gpurun_out/abc3/k${t}_o${o}_$i.log
      timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps ${STEPS:-100} --warmup 10 --tune 28=$t --orbit-step $o > $L 2>&1 || { echo "FAILED $t $o $i"; tail -3 $L; exit 1; }
      tail -1 $L | python3 -c "import json,sys; d=json.load(sys.stdin); print('knob28=$t orbit=$o round $i', round(d['value'],1), round(d['sequential']['value'],1), d['stages_ms'])"
    done
  done
done
