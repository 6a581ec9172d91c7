set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for X in 0 1 3 4 12; do
  O=gpurun_out/exp_$X; mkdir -p $O
  GSR_EXPERIMENT=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --inflight 1 --warm-ms 100 > $O/kt.log 2>&1 || exit 1
  python3 tools/summarize_prof.py $O > $O/summary.txt 2>&1
  echo "== X=$X"; grep -E "k_bin_(cols|rows)_scatter" $O/summary.txt
done
