# data-parallel tests incl. the bf16 graph mode (2 gloo ranks on one GPU)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dpbf.log 2>&1; rc=$?; echo "rc=$rc"; grep -h "PASS\|FAIL\|Error\|assert" gpurun_out/pytest_dpbf.log | head -20
exit $rc
