#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) over tools/bb_probe.py: config 3
# on a steady orbit with BUCKETS (knob 28), per-kernel means of the bucket-sort kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/bbpmc_${BUCKETS:-1}${KT_TAG:-}; mkdir -p $O
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE;FETCH_SIZE;WRITE_SIZE}"
for G in "${GROUPS_[@]}"; do
  T=$(echo $G | awk '{print $1}')
  BUCKETS=${BUCKETS:-1} FRAMES=${FRAMES:-40} timeout -k 10 120 rocprofv3 --pmc $G -d $O/pmc_$T -o pmc --output-format csv -- python3 tools/bb_probe.py > $O/pmc_$T.log 2>&1
  rc=$?; echo "pmc [$G] rc=$rc"; [ $rc = 0 ] || exit $rc
done
python3 tools/pmc_agg.py $O "${PMC_KERNELS:-k_b}" | tee $O/pmc_means.txt
find $O -name "*counter_collection.csv" -delete
