#!/bin/bash
# Round-2 first GPU session: environment probe, new GPU tests, full GPU suite,
# bench at 20 and 200 steps (steady-state check), 2-rank gloo bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2; stopping"; exit "$1";; esac; }
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}";
  timeout 30 rocm-smi --showpower --showclocks --showtemp --json 2>&1 | head -c 4000; echo;
  timeout 30 rocm-smi --showperflevel 2>&1 | head -20; } > gpurun_out/probe.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_path.py tests/test_gpu_multi_rank.py "tests/test_gpu_parity.py::test_viewer_link_binary_renders_like_oracle" -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -n 12 gpurun_out/pytest_new.log; fatal $rc pytest_new; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; fatal $rc bench20
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench200.log 2>&1
rc=$?; echo "bench200 rc=$rc"; fatal $rc bench200
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "bench gloo2 rc=$rc"; fatal $rc bench_gloo2
for f in bench20 bench200 bench_gloo2; do tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['n_gpus'], d['sequential']['value'], d['roofline']['avg_launch_ms'], d.get('cpu_baseline',{}).get('cores'))"; done
