set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_quant_step.py tests/test_gpu_plugin.py -k "quant or c5" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t10.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR|h max diff|RMSprop-amplified" gpurun_out/r5_t10.log | cut -c1-300 | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c5 > gpurun_out/r5prof/trace_c5_qx1.json 2> gpurun_out/r5prof/trace_c5_qx1.err
echo "trace rc=$?"; cat gpurun_out/r5prof/trace_c5_qx1.json | tr -d '\n' | cut -c1-900; echo
