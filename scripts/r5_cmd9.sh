set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_quant_step.py tests/test_gpu_configs.py tests/test_gpu_plugin.py tests/test_gpu_seq_graph.py tests/test_gpu_rnn.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t11.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR|output max diff|quantised h elements|RMSprop-amplified" gpurun_out/r5_t11.log | cut -c1-400 | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ex in 1 0 1 0; do
PKC_RNN_QH_EXACT=$ex timeout -k 10 300 python -u scripts/bench_seq.py --configs c5 --steps 12 --warmup 3 > gpurun_out/r5prof/c5b_exact$ex.log 2>&1
echo "c5 exact=$ex rc=$? $(grep '^{' gpurun_out/r5prof/c5b_exact$ex.log | cut -c1-260)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc5b -o run -- python3 scripts/bench_seq.py --configs c5 --steps 6 --warmup 2 > gpurun_out/r5prof/c5bprof.log 2>&1
echo "c5 prof rc=$?"; cp "$(find /tmp/pc5b -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/c5b_exact_kernel_stats.csv; head -6 gpurun_out/r5prof/c5_exact_kernel_stats.csv | cut -c1-160
