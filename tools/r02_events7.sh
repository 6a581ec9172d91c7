#!/bin/bash
# World-1 rehearsal diagnostic: one render_path call with and without per-frame completion events.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
run() {
  local port=$((29600 + RANDOM % 300))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $2 \
    > gpurun_out/rehearsal7_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal7_$1.log; exit $rc; }
  grep "nccl rehearsal" gpurun_out/rehearsal7_$1.log
}
for rep in 1 2; do
  run r16_$rep "--gather none --ring 16"
  run r8_$rep "--gather none --ring 8"
  run none$rep "--gather none"
done
