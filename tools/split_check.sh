#!/bin/bash
# Depth-split evidence in one call: its GPU tests, then an interleaved config-3 A/B of the
# split (default) against the split off (tools/ab_tunes.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/split
timeout -k 10 900 python -u -m pytest tests/test_gpu_depth_split.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/split/tests.log 2>&1
rc=$?; tail -28 gpurun_out/split/tests.log; [ $rc = 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} TUNES="${TUNES:-- 23=0}" BENCH_ARGS="${BENCH_ARGS:---config 3 --steps 100 --warmup 10}" bash tools/ab_tunes.sh
