set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_glds.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_glds.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
PKC_GEMM_GLDS=$v timeout -k 10 300 python bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4096.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b4096.log').read().strip().splitlines()[-1]); print('glds=$v B4096', d['value'], d['ms_per_step'])"
done
