#!/bin/bash
# World-1 RCCL rehearsal of the multi-GPU frame loop at several chunk sizes (frames per
# gather), interleaved with the no-gather loop: ROUNDS x (none, chunk c for c in CHUNKS).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/reh_chunks
for i in $(seq 1 ${ROUNDS:-2}); do
  for c in none ${CHUNKS:-8 16 32 64}; do
    if [ $c = none ]; then G="--gather none"; else G="--gather step --chunk $c"; fi
    timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 400)) tools/nccl_rehearsal.py $G ${REH_ARGS:---steps 512 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000} \
      > gpurun_out/reh_chunks/${c}_$i.log 2>&1
    rc=$?; grep "nccl rehearsal" gpurun_out/reh_chunks/${c}_$i.log | sed "s/^/[$c $i] /"
    case $rc in 0) ;; *) tail -5 gpurun_out/reh_chunks/${c}_$i.log; exit $rc;; esac
  done
done
