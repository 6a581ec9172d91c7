#!/bin/bash
# Kernel trace of the world-1 RCCL frame loop (what the per-step gathers launch and how long it runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/prof_gather
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 300))
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gather -o gt -- \
  python tools/nccl_rehearsal.py --steps 200 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 300 \
  > gpurun_out/prof_gather/run.log 2>&1
rc=$?; echo "rc=$rc"; grep "nccl rehearsal" gpurun_out/prof_gather/run.log; [ $rc = 0 ] || { tail -20 gpurun_out/prof_gather/run.log; exit $rc; }
find gpurun_out/prof_gather -name "*kernel_stats.csv" | head -3
