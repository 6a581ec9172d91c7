#!/bin/bash
# World-1 RCCL rehearsal at config-2 size with rank 0's gather slot aliased to its output
# (no local copy), against the same frames without gathers; then the multi-rank GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_multi_rank.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_mr5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_mr5.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
run() {
  local port=$((29600 + RANDOM % 300))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $2 \
    > gpurun_out/rehearsal5_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal5_$1.log; exit $rc; }
  grep "nccl rehearsal" gpurun_out/rehearsal5_$1.log
}
for rep in 1 2; do
  run alias$rep ""
  run nocalls$rep "--no-gather-calls"
  run nocalls16_$rep "--no-gather-calls --chunk 64"
  run none$rep "--gather none"
done
