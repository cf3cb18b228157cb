# LDS-DMA 128x128 body: GEMM parity tests, then large-M TF/s with and without it (PKC_GEMM_GLDS)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/pytest_glds.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/pytest_glds.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
PKC_GEMM_GLDS=$v timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_glds$v.log 2>&1 || exit $?
echo "glds=$v"; grep -v grouped gpurun_out/gemm_glds$v.log | grep "mlp\|square" | cut -c1-110
done
