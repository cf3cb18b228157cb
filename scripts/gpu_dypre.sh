# dL/dy slab presum before the BPTT loop: sequence parity tests, then C3/C4/C5/GRU with
# PKC_REC_DY_PRESUM=0 / 1 alternating (same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_quant_step.py tests/test_gpu_run_nn_parity.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dypre.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_dypre.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
PKC_REC_DY_PRESUM=$v timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4,c5,gru --steps 16 > gpurun_out/dypre_$v.log 2>&1 || exit $?
echo "presum=$v"; grep '^{' gpurun_out/dypre_$v.log | cut -c1-105
done
