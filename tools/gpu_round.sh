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
#   rehkt      kernel + memory-copy trace of the world-1 RCCL rehearsal, with per-chunk gathers
#              and without (rank env set directly: no launcher under the profiler)
#   ktab       kernel trace of the one-frame-at-a-time bench per knob setting (TUNES,
#              e.g. TUNES="19=0 19=1"; CONFIGS; KT_ARGS, e.g. "--orbit-step 0.25")
#              -> gpurun_out/kt_ab_<tag>/summary.txt
#   abtune     interleaved knob A/B in one process (tools/ab_path.py, AB_ARGS)
#   ablibs     interleaved A/B of two library builds            (tools/ab_libs.sh)
#
#   sh3        config 2 as BASELINE states it (SH degree 3): bench.py --sh3, 200 steps, then the
#              kernel trace and FETCH/WRITE PMC of its one-frame-at-a-time run -> prof_${TAG}_sh3
#   orbit      config 3 on a moving camera (--orbit-step 0.25; depth split on and off) beside the
#              fixed camera, twice interleaved -> bench_${TAG}_c3_{fixed,orbit,orbitoff}_{1,2}.log
#   stretch    kernel trace of the frames-in-flight bench and tools/blend_stretch.py: which
#              geometry kernels beside a blend lengthen it -> prof_${TAG}_stretch/stretch.txt
#
#   STEPS="suite smoke bench" TAG=r03 bash tools/gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-run}
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
slim() {   # drop the raw per-dispatch traces (gpurun brings back at most 64 MiB); keep stats + summaries
  find "$1" \( -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv" -o -name "*counter_collection.csv" \) -delete 2>/dev/null
  true
}
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
    # one frame at a time, headline frames only (the orbit / SH-3 objects' frames would mix
    # other views into the per-kernel means), like the bench's avg_launch_ms
    OUT=gpurun_out/prof_$TAG BENCH_ARGS=${BENCH_ARGS:---inflight 1 --no-orbit-line --no-sh3-line} SKIP_PMC=1 bash tools/profile.sh
    rc=$?; fatal $rc kt; [ $rc = 0 ] || exit $rc
    python3 tools/summarize_prof.py gpurun_out/prof_$TAG > gpurun_out/prof_$TAG/summary.txt 2>&1; head -30 gpurun_out/prof_$TAG/summary.txt
    slim gpurun_out/prof_$TAG ;;
  pmc)
    # PMC passes of the one-frame-at-a-time bench (BENCH_ARGS default --inflight 1), the
    # per-kernel means written as gpurun_out/pmc_$TAG.json (bench.py reads profiles/pmc_latest.json)
    OUT=gpurun_out/prof_$TAG BENCH_ARGS=${BENCH_ARGS:---inflight 1 --no-orbit-line --no-sh3-line} SKIP_KT=1 \
      PMC_GROUPS=${PMC_GROUPS:-"FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU"} \
      bash tools/profile.sh
    rc=$?; fatal $rc pmc; [ $rc = 0 ] || exit $rc
    python3 tools/summarize_prof.py gpurun_out/prof_$TAG --json gpurun_out/pmc_$TAG.json ${PMC_CONFIG:-2} \
      "rocprofv3 --pmc, separate passes, bench.py --steps 50 ${BENCH_ARGS:---inflight 1 --no-orbit-line --no-sh3-line}, $TAG"
    python3 tools/pmc_agg.py gpurun_out/prof_$TAG k_ > gpurun_out/prof_$TAG/pmc_means.txt 2>&1
    # with a kernel trace of the same TAG already there: the table with the PMC columns
    [ -f gpurun_out/prof_$TAG/kt/kt_kernel_stats.csv ] && \
      python3 tools/summarize_prof.py gpurun_out/prof_$TAG > gpurun_out/prof_$TAG/summary.txt 2>&1
    slim gpurun_out/prof_$TAG ;;
  rehearsal)
    for g in step none; do
      timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 400)) tools/nccl_rehearsal.py --gather $g ${REH_ARGS:---steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000} \
        > gpurun_out/rehearsal_${TAG}_$g.log 2>&1
      rc=$?; fatal $rc rehearsal; grep "nccl rehearsal" gpurun_out/rehearsal_${TAG}_$g.log; [ $rc = 0 ] || { tail -5 gpurun_out/rehearsal_${TAG}_$g.log; exit $rc; }
    done ;;
  rehkt)
    for g in step none; do
      O=gpurun_out/prof_reh_${TAG}_$g; mkdir -p $O
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 400)) \
        timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/kt -o kt --output-format csv -- \
        python3 tools/nccl_rehearsal.py --gather $g ${REH_ARGS:---steps 400 --gaussians 1000000 --W 1920 --H 1080 --warm-ms 1000} > $O/kt.log 2>&1
      rc=$?; echo "rehearsal trace $g rc=$rc"; fatal $rc rehkt; grep "nccl rehearsal" $O/kt.log; [ $rc = 0 ] || { tail -5 $O/kt.log; exit $rc; }
      python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; head -24 $O/summary.txt
      slim $O
    done ;;
  ktab)
    for t in ${TUNES:-19=0 19=1}; do
      tg=$(echo "$t" | tr '=,' '__'); O=gpurun_out/kt_ab_$tg; mkdir -p $O
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIGS:-2} --steps 60 --warmup 5 --no-cpu-baseline --no-sh3-line --no-orbit-line --inflight 1 --warm-ms 200 --tune "$t" ${KT_ARGS:-} > $O/kt.log 2>&1
      rc=$?; echo "tune $t kt rc=$rc"; fatal $rc ktab; [ $rc = 0 ] || exit $rc
      python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; echo "== $t"; head -16 $O/summary.txt
    done ;;
  abtune)
    timeout -k 10 600 python tools/ab_path.py ${AB_ARGS:-} > gpurun_out/abtune_$TAG.log 2>&1
    rc=$?; tail -20 gpurun_out/abtune_$TAG.log; fatal $rc abtune; [ $rc = 0 ] || exit $rc ;;
  ablibs)
    bash tools/ab_libs.sh; rc=$?; fatal $rc ablibs; [ $rc = 0 ] || exit $rc ;;
  sh3)
    timeout -k 10 300 python bench.py --config 2 --sh3 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_${TAG}_sh3.log 2>&1
    rc=$?; fatal $rc sh3; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_sh3.log; exit $rc; }
    line gpurun_out/bench_${TAG}_sh3.log sh3
    OUT=gpurun_out/prof_${TAG}_sh3 BENCH_ARGS="--sh3 --inflight 1" PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/profile.sh
    rc=$?; fatal $rc sh3prof; [ $rc = 0 ] || exit $rc
    python3 tools/summarize_prof.py gpurun_out/prof_${TAG}_sh3 > gpurun_out/prof_${TAG}_sh3/summary.txt 2>&1
    head -16 gpurun_out/prof_${TAG}_sh3/summary.txt; slim gpurun_out/prof_${TAG}_sh3 ;;
  orbit)
    for rep in 1 2; do
      for cam in fixed orbit orbitoff; do
        extra=""; [ $cam = orbit ] && extra="--orbit-step 0.25"; [ $cam = orbitoff ] && extra="--orbit-step 0.25 --tune 23=0"
        timeout -k 10 300 python bench.py --config 3 --steps 200 --warmup 20 --no-cpu-baseline $extra > gpurun_out/bench_${TAG}_c3_${cam}_$rep.log 2>&1
        rc=$?; fatal $rc orbit; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_c3_${cam}_$rep.log; exit $rc; }
        line gpurun_out/bench_${TAG}_c3_${cam}_$rep.log "config3 $cam"
      done
    done ;;
  stretch)
    O=gpurun_out/prof_${TAG}_stretch; mkdir -p $O
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --config ${CONFIGS:-2} --steps 200 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/kt.log 2>&1
    rc=$?; echo "stretch trace rc=$rc"; fatal $rc stretch; [ $rc = 0 ] || { tail -5 $O/kt.log; exit $rc; }
    python3 tools/blend_stretch.py $O > $O/stretch.txt 2>&1; cat $O/stretch.txt
    python3 tools/overlap.py $O > $O/overlap.txt 2>&1 || true
    slim $O ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
