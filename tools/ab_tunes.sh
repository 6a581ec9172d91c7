#!/bin/bash
# Interleaved A/B of knob settings through bench.py --tune: ROUNDS x (each of TUNES) bench
# runs, each in its own process.  TUNES: space-separated --tune values, "-" = defaults
# (e.g. TUNES="- 23=0"); BENCH_ARGS: the bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abtunes
for i in $(seq 1 ${ROUNDS:-2}); do
  for T in ${TUNES:--}; do
    tag=$(echo "$T" | tr '=,' '__')
    log=gpurun_out/abtunes/${tag}_$i.log
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 100 --warmup 10} \
        $([ "$T" = - ] || echo --tune $T) > $log 2>&1 || { echo "FAILED $T $i"; tail -3 $log; exit 1; }
    tail -1 $log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$T', $i, d['value'], 'seq', d['sequential']['value'], 'blend', d['roofline']['avg_launch_ms'], d['stages_ms'], d.get('depth_split'), d['image_mean'])"
  done
done
