# Slab sums in their own grouped instance: tests, then B = 128 / 1024 / 4096 steps
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_b4k.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_b4k.log
[ $rc -eq 0 ] || exit $rc
for b in 128 4096 1024 128; do
st=200; [ $b -gt 128 ] && st=30
timeout -k 10 300 python bench.py --batch $b --steps $st --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b$b.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b$b.log').read().strip().splitlines()[-1]); print('B$b', d['value'], d['ms_per_step'])"
done
