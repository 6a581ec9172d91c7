#!/bin/bash
# GPU suite + smoke + a 200-step bench (every GPU step time-limited; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
TAG=${TAG:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 4 gpurun_out/pytest_$TAG.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log; fatal $rc smoke; [ $rc = 0 ] || exit $rc
for c in ${BENCH_CONFIGS:-2}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-200} --warmup 20 ${BENCH_EXTRA:---no-cpu-baseline} > gpurun_out/bench_${TAG}_c$c.log 2>&1
  rc=$?; fatal $rc bench; [ $rc = 0 ] || exit $rc
  tail -1 gpurun_out/bench_${TAG}_c$c.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config', $c, d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['stages_ms'])"
done
