# BatchNorm finalize workgroup width A/B: a library built with -DPKC_FIN_COLS=4 vs the default 16
# (build the variant as pkc/libpkc_fin16.so in the round-2 run; kept for the record)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_run_nn_parity.py tests/test_gpu_seq.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fin.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_fin.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in libpkc.so libpkc_fin16.so; do
PKC_LIB=$PWD/pytorch-kaldi-cgs_amd/pkc/$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/fin_$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/fin_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['batch_sweep_frames_per_s'])"
done
done
