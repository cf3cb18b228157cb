# small-batch BatchNorm kernels with 4-column workgroups (libpkc built with -DPKC_DENSE_FG=1, loaded
# through PKC_LIB) vs the 8-column default: MLP parity tests with it, then C2 alternating (same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PKC_LIB=$PWD/pytorch-kaldi-cgs_amd/pkc/libpkc_fg1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fg1.log 2>&1 || { tail -20 gpurun_out/pytest_fg1.log; exit 1; }
tail -1 gpurun_out/pytest_fg1.log
for r in 1 2; do
for v in libpkc.so libpkc_fg1.so; do
PKC_LIB=$PWD/pytorch-kaldi-cgs_amd/pkc/$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/fg1_$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/fg1_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['batch_sweep_frames_per_s'])"
done
done
