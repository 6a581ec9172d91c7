#!/bin/bash
# End-of-round check of HEAD: GPU suite, smoke, the driver's default bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_last.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 2 gpurun_out/pytest_last.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_last.log; fatal $rc smoke; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_last_default.log 2>&1
rc=$?; fatal $rc bench; [ $rc = 0 ] || { tail -5 gpurun_out/bench_last_default.log; exit $rc; }
tail -1 gpurun_out/bench_last_default.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('default', d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
