#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel trace + stats, then each PMC
# counter group in its own pass (never combined with other trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
B="bench.py --steps ${BENCH_STEPS:-50} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-}"
[ "${SKIP_KT:-0}" = 1 ] || timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 $B > "$OUT/kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; fatal $rc kt
# counter groups separated by ';' (each group = one pass)
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE}"
for G in "${GROUPS_[@]}"; do
  TAG=$(echo $G | awk '{print $1}')
  timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 --pmc $G -d "$OUT/pmc_$TAG" -o pmc --output-format csv -- python3 $B > "$OUT/pmc_$TAG.log" 2>&1
  rc=$?; echo "pmc [$G] rc=$rc"; fatal $rc "pmc $G"
done
find "$OUT" -name "*.csv" | head -20
