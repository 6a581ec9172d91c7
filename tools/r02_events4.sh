#!/bin/bash
# World-1 RCCL rehearsal at config-2 size: host enqueue time of the gather loop vs the GPU time.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
run() {  # tag, env, args
  local port=$((29600 + RANDOM % 300))
  env $2 timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $3 \
    > gpurun_out/rehearsal4_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal4_$1.log; exit $rc; }
  grep "nccl rehearsal" gpurun_out/rehearsal4_$1.log
}
for rep in 1 2; do
  run base$rep "X=1" ""
  run chunk32_$rep "X=1" "--chunk 32"
  run none$rep "X=1" "--gather none"
done
