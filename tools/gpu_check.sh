#!/bin/bash
# One GPU-box session: GPU tests, smoke, short bench.  Every GPU step has its
# own time limit; a fault / abort / timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
STEPS=${STEPS:-100}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 3 gpurun_out/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 5 gpurun_out/bench.log; fatal $rc bench
