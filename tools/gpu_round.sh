#!/bin/bash
# The one GPU-box driver for round evidence.  STEPS (space-separated, in order) picks
# what runs; every GPU step has its own time limit and a failure stops the script.
#
#   suite      pytest -m gpu (the driver's GPU tier)            -> gpurun_out/pytest_$TAG.log
#   smoke      __graft_entry__.smoke()                          -> gpurun_out/smoke_$TAG.log
#   bench      the driver's command: bench.py --steps 20 --warmup 5 (CPU baseline on)
#   bench200   bench.py --config $c --steps 200 for c in $CONFIGS (default 2)
#   kt         rocprofv3 kernel trace + stats of the bench    (tools/profile.sh, SKIP PMC)
#   pmc        the PMC passes of the same command              (tools/profile.sh, PMC only)
#   rehearsal  RCCL rehearsal of the multi-GPU loop at world 1 (tools/nccl_rehearsal.py),
#              with per-chunk gathers and without gathers (REH_ARGS)
#   ktab       kernel trace of the one-frame-at-a-time bench per knob setting (TUNES,
#              e.g. TUNES="19=0 19=1"; CONFIGS) -> gpurun_out/kt_ab_<tag>/summary.txt
#   abtune     interleaved knob A/B in one process (tools/ab_path.py, AB_ARGS)
#   ablibs     interleaved A/B of two library builds            (tools/ab_libs.sh)
#
#   STEPS="suite smoke bench" TAG=r03 bash tools/gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-run}
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
line() {   # summary of a bench JSON line
  tail -1 "$1" | python3 -c "import json,sys; d=json.load(sys.stdin); print('$2', d['value'], 'seq', d['sequential']['value'], 'blend', d['roofline']['avg_launch_ms'], 'inflight blend', d['roofline']['avg_launch_ms_inflight'], 'stages', d['stages_ms'], 'cpu', d.get('cpu_baseline', {}).get('value'))"
}
for step in ${STEPS:-suite smoke bench}; do
  case $step in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
    rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 3 gpurun_out/pytest_$TAG.log; fatal $rc pytest; [ $rc = 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log; fatal $rc smoke; [ $rc = 0 ] || exit $rc ;;
  bench)
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_default.log 2>&1
    rc=$?; fatal $rc bench; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_default.log; exit $rc; }
    line gpurun_out/bench_${TAG}_default.log default ;;
  bench200)
    for c in ${CONFIGS:-2}; do
      timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}_c$c.log 2>&1
      rc=$?; fatal $rc bench200; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_c$c.log; exit $rc; }
      line gpurun_out/bench_${TAG}_c$c.log config$c
    done ;;
  kt)
    OUT=gpurun_out/prof_$TAG SKIP_PMC=1 bash tools/profile.sh
    rc=$?; fatal $rc kt; [ $rc = 0 ] || exit $rc
    python3 tools/summarize_prof.py gpurun_out/prof_$TAG > gpurun_out/prof_$TAG/summary.txt 2>&1; head -30 gpurun_out/prof_$TAG/summary.txt ;;
  pmc)
    OUT=gpurun_out/prof_$TAG SKIP_KT=1 bash tools/profile.sh
    rc=$?; fatal $rc pmc; [ $rc = 0 ] || exit $rc ;;
  rehearsal)
    for g in step none; do
      timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 400)) tools/nccl_rehearsal.py --gather $g ${REH_ARGS:---steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000} \
        > gpurun_out/rehearsal_${TAG}_$g.log 2>&1
      rc=$?; fatal $rc rehearsal; grep "nccl rehearsal" gpurun_out/rehearsal_${TAG}_$g.log; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal_${TAG}_$g.log; exit $rc; }
    done ;;
  ktab)
    for t in ${TUNES:-19=0 19=1}; do
      tg=$(echo "$t" | tr '=,' '__'); O=gpurun_out/kt_ab_$tg; mkdir -p $O
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIGS:-2} --steps 60 --warmup 5 --no-cpu-baseline --inflight 1 --warm-ms 200 --tune "$t" > $O/kt.log 2>&1
      rc=$?; echo "tune $t kt rc=$rc"; fatal $rc ktab; [ $rc = 0 ] || exit $rc
      python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; echo "== $t"; head -16 $O/summary.txt
    done ;;
  abtune)
    timeout -k 10 600 python tools/ab_path.py ${AB_ARGS:-} > gpurun_out/abtune_$TAG.log 2>&1
    rc=$?; tail -20 gpurun_out/abtune_$TAG.log; fatal $rc abtune; [ $rc = 0 ] || exit $rc ;;
  ablibs)
    bash tools/ab_libs.sh; rc=$?; fatal $rc ablibs; [ $rc = 0 ] || exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
