#!/bin/bash
# Interleaved A/B of two environment settings of the same build: ROUNDS x (A, B) bench
# runs, each in its own process.  ENV_A / ENV_B: e.g. "GSR_BLEND_EXP=0" and "".
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abenv
for i in $(seq 1 ${ROUNDS:-3}); do
  for L in A B; do
    if [ $L = A ]; then E=${ENV_A:-}; else E=${ENV_B:-}; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 100 --warmup 10} > gpurun_out/abenv/${L}_$i.log 2>&1 || { echo "FAILED $L $i"; tail -3 gpurun_out/abenv/${L}_$i.log; exit 1; }
    tail -1 gpurun_out/abenv/${L}_$i.log | python3 -c "import json,sys; d=json.load(sys.stdin); c=d['blend_counters']; print('$L', $i, d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['stages_ms'], 'reblend', c.get('reblended_blocks'), c.get('suspect_pixels'))"
  done
done
