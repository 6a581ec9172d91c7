#!/bin/bash
# Gather-done wait events + no fork in the RCCL frame loop: GPU path / multi-rank tests, then the
# world-1 rehearsal (per-step gathers) against the same frames without gathers.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_multi_rank.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_ev9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_ev9.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
run() {
  local port=$((29600 + RANDOM % 300))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $2 \
    > gpurun_out/rehearsal9_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal9_$1.log; exit $rc; }
  echo "$1: $(grep 'nccl rehearsal' gpurun_out/rehearsal9_$1.log | grep -o '[0-9.]* frames/s\|bit-exact\|FAILED' | tr '\n' ' ')"
}
for rep in 1 2; do
  run step$rep ""
  run step3_$rep "--inflight 3"
  run step16_$rep "--chunk 16"
  run none$rep "--gather none"
done
