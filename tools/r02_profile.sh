#!/bin/bash
# Round-2 profile of the bench workload (config 2 unless CONFIG is set): kernel trace
# + stats, then PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction / cycle counters),
# each in its own run; summaries into gpurun_out/prof.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export STEPS=${STEPS:-50}
export BENCH_ARGS="--config ${CONFIG:-2} --inflight 1 --warm-ms 300 ${EXTRA:-}"
export PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
bash tools/profile.sh || exit $?
python3 tools/summarize_prof.py gpurun_out/prof > gpurun_out/prof/summary.txt
python3 tools/summarize_prof.py gpurun_out/prof --json gpurun_out/prof/pmc.json ${CONFIG:-2} "rocprofv3 --pmc, separate passes, bench.py --steps $STEPS --inflight 1, round 2"
grep "^{\"metric\"" gpurun_out/prof/kt.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench under profiler', d['value'], d['roofline']['avg_launch_ms'])"
