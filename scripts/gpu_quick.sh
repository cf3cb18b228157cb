set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q --timeout 200 -p no:cacheprovider > gpurun_out/pytest_mlp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_mlp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_prof.sh
