# 16-row recurrent step tiles (2B <= 16): parity tests, then C3/C5 throughput A/B
# (PKC_RNN_ROWS16=0/1, alternating, same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_quant_step.py tests/test_gpu_run_nn_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r16.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_r16.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
PKC_RNN_ROWS16=$v timeout -k 10 300 python scripts/bench_seq.py --configs c3,c5 --steps 20 > gpurun_out/r16_$v.log 2>&1 || exit $?
echo "rows16=$v"; grep '^{' gpurun_out/r16_$v.log | cut -c1-160
done
