#!/bin/bash
# GPU suite on the working-tree build, then interleaved A/B (HEAD vs working tree) on configs 3 and 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_pre.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 3 gpurun_out/pytest_pre.log; [ $rc = 0 ] || exit $rc
BENCH_ARGS="--config 3 --steps 100 --warmup 10 --warm-ms 500" ROUNDS=3 bash tools/ab_libs.sh || exit 1
BENCH_ARGS="--config 2 --steps 200 --warmup 10 --warm-ms 500" ROUNDS=3 bash tools/ab_libs.sh || exit 1
