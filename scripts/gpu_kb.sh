# Kernel micro-benchmarks (graph-replayed per-launch times at the C2 shapes) + large-M GEMM TF/s
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kbench.py "$@" > gpurun_out/kbench.log 2>&1 || exit $?
cat gpurun_out/kbench.log
timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gemm_bench.log
