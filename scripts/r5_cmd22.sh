set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_seq.py tests/test_gpu_seq_graph.py tests/test_gpu_configs.py -k "persist or ligru or bf16 or c3" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t31.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|T <= " gpurun_out/r5_t31.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u scripts/bench_seq.py --configs c3 --prec bf16 --steps 8 --warmup 2 > gpurun_out/r5prof/c3b_la2.log 2>&1
echo "c3 bf16 rc=$? $(grep '^{' gpurun_out/r5prof/c3b_la2.log | cut -c150-260)"
done
