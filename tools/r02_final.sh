#!/bin/bash
# Round-2 numbers of record: the driver's default bench line, 200-step benches of configs
# 2 / 3 / 5, then the kernel trace + PMC profile of config 2 (tools/r02_profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
TAG=${TAG:-final}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_default.log 2>&1
rc=$?; fatal $rc bench_default; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_default.log; exit $rc; }
tail -1 gpurun_out/bench_${TAG}_default.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('default', d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['cpu_baseline'])"
for c in ${CONFIGS:-2 3 5}; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_${TAG}_c$c.log 2>&1
  rc=$?; fatal $rc bench$c; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_c$c.log; exit $rc; }
  tail -1 gpurun_out/bench_${TAG}_c$c.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config', $c, d['value'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d['stages_ms'])"
done
[ "${PROFILE:-1}" = 1 ] && bash tools/r02_profile.sh
