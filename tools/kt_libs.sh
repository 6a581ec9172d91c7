set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
for L in N S N S; do
  O=gpurun_out/kt_lib_$L; mkdir -p $O
  GSR_LIBRARY=$PWD/gaussianrenderer_amd/lib/ab/libgsr_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config 3 --steps 40 --warmup 5 --no-cpu-baseline --no-sh3-line --inflight 1 --warm-ms 200 --tune 23=0 > $O/kt.log 2>&1 || { echo FAIL $L; tail -5 $O/kt.log; exit 1; }
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1; echo "== $L"; grep "radix_down\|radix_up" $O/summary.txt
  tail -1 $O/kt.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$L', d['value'], d['sequential']['value'], d['stages_ms'])"
done
