#!/bin/bash
# Interleaved A/B of builds of libgsr.so on one box: ROUNDS x (each of LIBS, default "A B") runs
# of the bench (BENCH_ARGS), each in its own process with GSR_LIBRARY pointing at the build.
# Builds: gaussianrenderer_amd/lib/ab/libgsr_<L>.so (A and B made by tools/ab_build.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for i in $(seq 1 ${ROUNDS:-3}); do
  for L in ${LIBS:-A B}; do
    GSR_LIBRARY=$PWD/gaussianrenderer_amd/lib/ab/libgsr_$L.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 100 --warmup 10} > gpurun_out/ab/${L}_$i.log 2>&1 || { echo "FAILED $L $i"; tail -3 gpurun_out/ab/${L}_$i.log; exit 1; }
    tail -1 gpurun_out/ab/${L}_$i.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', $i, d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['stages_ms'])"
  done
done
