# 8-wave recurrent step tiles: parity (PKC_RNN_WAVES=8) on the sequence tests, then a same-run A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PKC_RNN_WAVES=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_waves.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_waves.log
[ $rc -eq 0 ] || exit $rc
for w in 4 8 4 8; do
PKC_RNN_WAVES=$w timeout -k 10 300 python scripts/bench_seq.py --configs c4,c5,gru --steps 10 > gpurun_out/seq_w$w.log 2>&1 || exit $?
echo "waves=$w"; grep '^{' gpurun_out/seq_w$w.log | cut -c1-160
done
