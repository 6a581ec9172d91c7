#!/bin/bash
# Interleaved lanes A/B on the final code: bench config 2, 200 steps, --inflight 4 / 5 / 6.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for F in 4 5 6; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --warm-ms 500 --no-cpu-baseline --inflight $F > gpurun_out/lanes_${F}_$i.log 2>&1 || { echo "FAILED $F $i"; tail -3 gpurun_out/lanes_${F}_$i.log; exit 1; }
    tail -1 gpurun_out/lanes_${F}_$i.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('F=$F', $i, d['value'], d['sequential']['value'])"
  done
done
