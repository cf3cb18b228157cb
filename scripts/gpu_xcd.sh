# XCD-aware tile order of the standalone 128x128 launches: GEMM tests, then same-run A/B of the
# large-M matmuls and the B = 4096 / 1024 steps (PKC_GEMM_XCD=0/1)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/pytest_xcd.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -2 gpurun_out/pytest_xcd.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
PKC_GEMM_XCD=$v timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_xcd$v.log 2>&1 || exit $?
echo "xcd=$v"; grep -v grouped gpurun_out/gemm_xcd$v.log | grep "mlp\|square\|c4" | cut -c1-100
done
for v in 0 1 0 1; do
PKC_GEMM_XCD=$v timeout -k 10 300 python bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4096.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b4096.log').read().strip().splitlines()[-1]); print('xcd=$v B4096', d['value'], d['ms_per_step'])"
done
