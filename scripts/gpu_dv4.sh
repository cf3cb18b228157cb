# 16-byte large-M BatchNorm kernels: the GPU tests that run them (kernels, MLP at B >= 1024, run_nn
# lifecycle, sequence engines, DP), then B = 4096 / 1024 and C3/C4 with PKC_DENSE_V4 = 0 / 1
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_run_nn_parity.py tests/test_gpu_seq.py tests/test_gpu_rnn.py tests/test_gpu_configs.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dv4.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_dv4.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
PKC_DENSE_V4=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/dv4_$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/dv4_$v.log').read().strip().splitlines()[-1]); print('v4=$v', d['value'], d['batch_sweep_frames_per_s'])"
done
for v in 0 1; do
PKC_DENSE_V4=$v timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4,c5 --steps 10 > gpurun_out/dv4seq_$v.log 2>&1 || exit $?
echo "v4=$v"; grep '^{' gpurun_out/dv4seq_$v.log | cut -c1-100
done
