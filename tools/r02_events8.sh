#!/bin/bash
# World-1 rehearsal diagnostic: the chunked loop without gather calls, join per chunk vs frame events + no join.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
run() {
  local port=$((29600 + RANDOM % 300))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $2 \
    > gpurun_out/rehearsal8_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal8_$1.log; exit $rc; }
  echo "$1: $(grep 'nccl rehearsal' gpurun_out/rehearsal8_$1.log | sed 's/.*aggregate//')"
}
for rep in 1 2; do
  run nofork64_$rep "--no-gather-calls --no-fork --chunk 64"
  run nofork8_$rep "--no-gather-calls --no-fork --chunk 8"
  run nojoin64_$rep "--no-gather-calls --chunk 64"

  run none$rep "--gather none"
done
