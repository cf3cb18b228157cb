set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_plugin.py tests/test_gpu_seq.py tests/test_gpu_quant_step.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t8.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR|T <= 8|outliers \(count" gpurun_out/r5_t8.log | cut -c1-600 | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseqb -o run -- python3 scripts/bench_seq.py --configs c3 --steps 6 --warmup 2 --prec bf16 > gpurun_out/r5prof/seqprof8_bf16.log 2>&1
echo "seq_prof rc=$?"; grep '^{' gpurun_out/r5prof/seqprof8_bf16.log | cut -c1-330; cp "$(find /tmp/pseqb -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/seq8_bf16_kernel_stats.csv; head -4 gpurun_out/r5prof/seq8_bf16_kernel_stats.csv | cut -c1-150
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c5 > gpurun_out/r5prof/trace_c5.json 2> gpurun_out/r5prof/trace_c5.err
echo "trace rc=$?"; cat gpurun_out/r5prof/trace_c5.json; tail -3 gpurun_out/r5prof/trace_c5.err
