set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_mlp.py tests/test_gpu_seq.py tests/test_gpu_plugin.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t5.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR|T <= 8|step 0: post" gpurun_out/r5_t5.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_seq.py --configs c3 --steps 8 --warmup 2 --prec bf16 > gpurun_out/r5prof/seq5_bf16.log 2>&1
echo "seq rc=$?"; grep '^{' gpurun_out/r5prof/seq5_bf16.log | cut -c1-330
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseqb -o run -- python3 scripts/bench_seq.py --configs c3 --steps 6 --warmup 2 --prec bf16 > gpurun_out/r5prof/seqprof5_bf16.log 2>&1
echo "seq_prof rc=$?"; cp "$(find /tmp/pseqb -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/seq5_bf16_kernel_stats.csv; head -6 gpurun_out/r5prof/seq5_bf16_kernel_stats.csv | cut -c1-150
