set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile_depth.py tests/test_gpu_parity.py tests/test_gpu_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -25 gpurun_out/t1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_tds.log 2>&1; rc=$?; tail -1 gpurun_out/bench_tds.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['sequential'], d['stages_ms'], d['roofline']['avg_launch_ms'], d['roofline']['avg_launch_ms_inflight'], d['depth_passes'])"; exit $rc
