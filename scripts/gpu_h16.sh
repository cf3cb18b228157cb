# bf16 operand storage (PKC_PREC_BF16IN matmuls): equality with bf16 staging, the MLP GPU tests,
# then the C2 step and the batch sweep with PKC_BF16_STORE = 0 / 1 alternating (same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_h16.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_h16.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
PKC_BF16_STORE=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/bh16_$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bh16_$v.log').read().strip().splitlines()[-1]); print('store=$v', d['value'], d['ms_per_step'], d.get('batch_sweep'), d['roofline'])"
done
