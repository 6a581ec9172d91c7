#!/bin/bash
# World-1 RCCL rehearsal at config-2 size: lanes x (frame events / join per chunk), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
for rep in 1 2; do
  for cfg in "--inflight 4 --warm-ms 1000" "--inflight 4 --warm-ms 1000 --gather none" "--inflight 4 --warm-ms 1000 --no-overlap" "--inflight 3 --warm-ms 1000"; do
    port=$((29600 + RANDOM % 300))
    tag=$(echo "$cfg" | tr -d " -")
    timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 $cfg \
      > gpurun_out/rehearsal2_${rep}_$tag.log 2>&1
    rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal2_${rep}_$tag.log; exit $rc; }
    grep "nccl rehearsal" gpurun_out/rehearsal2_${rep}_$tag.log
  done
done
