# small-batch BatchNorm forms (8 columns for N >= 512, 16 below, M <= 128): dense kernel tests,
# the run_nn lifecycle tests, then the C2 bench line
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_run_nn_parity.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_m128.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_m128.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/m128.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/m128.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
