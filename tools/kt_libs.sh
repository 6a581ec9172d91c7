#!/bin/bash
# Kernel traces of several builds of libgsr.so on one box, interleaved: for each round and
# each LIBS entry L, rocprofv3 --kernel-trace --stats of one bench run with
# GSR_LIBRARY=gaussianrenderer_amd/lib/ab/libgsr_$L.so (BENCH_ARGS), then its summary and
# bench line.  -> gpurun_out/kt_lib_<L>_<round>/
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in ${LIBS:-A B}; do
    O=gpurun_out/kt_lib_${L}_$r; mkdir -p $O
    GSR_LIBRARY=$PWD/gaussianrenderer_amd/lib/ab/libgsr_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py ${BENCH_ARGS:---config 3 --steps 40 --warmup 5 --no-cpu-baseline --no-sh3-line --inflight 1 --warm-ms 200 --tune 23=0} > $O/kt.log 2>&1 || { echo FAIL $L; tail -5 $O/kt.log; exit 1; }
    python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; echo "== $L round $r"; sed -n 3,16p $O/summary.txt
    grep '^{' $O/kt.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', d['value'], d['sequential']['value'], d['stages_ms'])" || true
    find $O -name "*kernel_trace.csv" -delete
  done
done
