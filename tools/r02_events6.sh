#!/bin/bash
# World-1 RCCL rehearsal: output-buffer footprint (chunk size: 2 sets x chunk buffers of 24.9 MB)
# with and without the gather calls, against one render_path call over a ring of 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
run() {
  local port=$((29600 + RANDOM % 300))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port tools/nccl_rehearsal.py --steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000 $2 \
    > gpurun_out/rehearsal6_$1.log 2>&1
  local rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal6_$1.log; exit $rc; }
  grep "nccl rehearsal" gpurun_out/rehearsal6_$1.log
}
for rep in 1 2; do
  run nc2_$rep "--no-gather-calls --chunk 2"
  run nc4_$rep "--no-gather-calls --chunk 4"
  run g2_$rep "--chunk 2"
  run g4_$rep "--chunk 4"
  run none$rep "--gather none"
done
