#!/bin/bash
# GPU check after a kernel change: full GPU suite, smoke, benches (configs in BENCH_CONFIGS),
# optional extra command (EXTRA_CMD) — every GPU step time-limited, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
TAG=${TAG:-run}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 4 gpurun_out/pytest_$TAG.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
fi
for c in ${BENCH_CONFIGS:-2}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/bench_${TAG}_c$c.log 2>&1
  rc=$?; fatal $rc bench; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_c$c.log; exit $rc; }
  tail -1 gpurun_out/bench_${TAG}_c$c.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config', $c, d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['stages_ms'])"
done
if [ -n "${EXTRA_CMD:-}" ]; then
  timeout -k 10 300 bash -c "$EXTRA_CMD" > gpurun_out/extra_$TAG.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -n 20 gpurun_out/extra_$TAG.log; fatal $rc extra
fi
