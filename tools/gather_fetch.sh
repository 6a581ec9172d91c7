set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gf
timeout -k 10 60 ./tools/microbench/gather_fetch > gpurun_out/gf/time.csv 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gf/pmc -o pmc --output-format csv -- ./tools/microbench/gather_fetch > gpurun_out/gf/pmc.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/gf/pmc2 -o pmc --output-format csv -- ./tools/microbench/gather_fetch > gpurun_out/gf/pmc2.log 2>&1
echo rc2=$?
find gpurun_out/gf -name "*.csv"
