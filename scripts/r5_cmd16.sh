set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
PKC_RNN_QH_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_quant_step.py "tests/test_gpu_configs.py" -k "quant or c5" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t16.log 2>&1
rc=$?; echo "tests(16 waves) rc=$rc"; grep -E "passed|failed|^FAILED|h max diff" gpurun_out/r5_t16.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in 16 8 16 8; do
PKC_RNN_QH_WAVES=$w timeout -k 10 300 python -u scripts/bench_seq.py --configs c5 --steps 12 --warmup 3 > gpurun_out/r5prof/c5w$w.log 2>&1
echo "c5 waves=$w rc=$? $(grep '^{' gpurun_out/r5prof/c5w$w.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(round(d['us_per_time_step_per_layer_fwd_bwd'],3), round(d['frames_per_s']))")"
done
