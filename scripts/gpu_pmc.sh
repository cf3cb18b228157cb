# HBM traffic of the bench's dominant launch: two rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950) over `bench.py --pmc-replay N`, which replays only
# that launch; summarised by scripts/pmc_summary.py into gpurun_out/pmc_traffic.json
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
N=20
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o f -- python3 bench.py --pmc-replay $N --pmc-kernel ${PMC_KERNEL:-pkc_gemm_grouped} > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o w -- python3 bench.py --pmc-replay $N --pmc-kernel ${PMC_KERNEL:-pkc_gemm_grouped} > gpurun_out/pmc/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc $N > gpurun_out/pmc_traffic.json
cat gpurun_out/pmc_traffic.json
