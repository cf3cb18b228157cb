# Parity + A/B of the fp32 LDS-swizzle GEMM build (pkc/libpkc_swz.so) against the default build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_swz.so
PKC_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_rnn.py tests/test_gpu_seq.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/swz_tests.log 2>&1
rc=$?; tail -2 gpurun_out/swz_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_libab.sh "" _swz || exit $?
timeout -k 10 300 python scripts/bench_seq.py > gpurun_out/seq_def.log 2>&1 || exit $?
PKC_LIB=$V timeout -k 10 300 python scripts/bench_seq.py > gpurun_out/seq_swz.log 2>&1 || exit $?
PKC_LIB=$V timeout -k 10 200 python scripts/kbench.py big > gpurun_out/kb_big_swz.log 2>&1 || exit $?
grep -h '^{' gpurun_out/seq_def.log gpurun_out/seq_swz.log | cut -c1-110
grep big gpurun_out/kb_big_swz.log
