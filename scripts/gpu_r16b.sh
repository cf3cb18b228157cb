# 16-row recurrent step tiles for every cell: parity tests, then the sequence configs with
# PKC_RNN_ROWS16 = 0 (32-row tiles), 16 (default), 32 (16-row tiles also for C4's 2B = 32)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_quant_step.py tests/test_gpu_run_nn_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r16.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_r16.log
[ $rc -eq 0 ] || exit $rc
PKC_RNN_ROWS16=64 timeout -k 10 500 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r16_64.log 2>&1
rc=$?; echo "tests (all 16-row) rc=$rc"; tail -3 gpurun_out/pytest_r16_64.log
[ $rc -eq 0 ] || exit $rc
for v in 0 16 32 0 16 32; do
PKC_RNN_ROWS16=$v timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4,c5,gru --steps 16 > gpurun_out/r16b_$v.log 2>&1 || exit $?
echo "rows16=$v"; grep '^{' gpurun_out/r16b_$v.log | cut -c1-110
done
