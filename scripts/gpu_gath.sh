# 16-byte batch gather: kernel + MLP tests, then C2 (same box, this build vs the committed A/B numbers)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_run_nn_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gath.log 2>&1; rc=$?
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in 1; do
PKC_X=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/gath_$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/gath_$v.log').read().strip().splitlines()[-1]); print('vec=$v', d['value'], d['ms_per_step'], d.get('posterior_max_rel_err'))"
done
done
