#!/bin/bash
# Steady-state check: the driver's short bench (20 steps) against a 200-step run, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
for tag in a b c; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/steady20_$tag.log 2>&1
  rc=$?; fatal $rc steady20; [ $rc = 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/steady200.log 2>&1
rc=$?; fatal $rc steady200; [ $rc = 0 ] || exit $rc
for f in steady20_a steady20_b steady20_c steady200; do tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['roofline']['avg_launch_ms_inflight'], d['sustained_warmup']['frames'])"; done
