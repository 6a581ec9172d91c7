#!/bin/bash
# Per-frame events without the exit join (gsr_render_path_ex): GPU path tests, then the
# world-1 RCCL rehearsal at config-2 size with and without the per-chunk join, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_multi_rank.py -x -q -p no:cacheprovider \
  --timeout 150 --timeout-method thread > gpurun_out/pytest_events.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_events.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for mode in "" "--no-overlap"; do
    port=$((29600 + RANDOM % 300))
    timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port tools/nccl_rehearsal.py --steps 200 --gaussians 1000000 --W 1920 --H 1080 --chunk 8 $mode \
      > gpurun_out/rehearsal_${rep}${mode}.log 2>&1
    rc=$?; fatal $rc rehearsal; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal_${rep}${mode}.log; exit $rc; }
    grep "nccl rehearsal" gpurun_out/rehearsal_${rep}${mode}.log
  done
done
