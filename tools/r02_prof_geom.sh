#!/bin/bash
# PMC passes over the config-3 bench (geometry kernels): SQ instruction, stall and LDS
# counters plus FETCH/WRITE, each group in its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profg
timeout -k 10 60 rocprofv3 -L > gpurun_out/profg/counters.txt 2>&1 || true
export STEPS=${STEPS:-20}
export BENCH_ARGS="--config ${CONFIG:-3} --inflight 1 --warm-ms 200"
export PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY;SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;FETCH_SIZE;WRITE_SIZE"
export SKIP_KT=0 PMC_TIMEOUT=300
OUT=gpurun_out/profg bash tools/profile.sh || exit $?
python3 tools/summarize_prof.py gpurun_out/profg > gpurun_out/profg/summary.txt 2>&1
python3 tools/pmc_agg.py gpurun_out/profg k_ > gpurun_out/profg/pmc_agg.txt 2>&1 || true
