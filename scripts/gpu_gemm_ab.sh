# New-GEMM check: big-tile parity tests, the 64x64 vs 128x128 A/B, and the B=4096 MLP step
# profile (kernel stats only).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out /tmp/b4k
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/pytest_big.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/pytest_big.log
[ $rc -eq 0 ] || exit $rc
PKC_GEMM_BIG=0 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_ab0.log 2>&1 || exit $?
PKC_GEMM_BIG=1 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_ab1.log 2>&1 || exit $?
tail -1 gpurun_out/gemm_ab0.log; tail -1 gpurun_out/gemm_ab1.log
for b in 0 1; do
PKC_GEMM_BIG=$b timeout -k 10 300 python bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k_$b.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/b4k_$b.log').read().strip().splitlines()[-1]); print('B4096 big=$b', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b4k -o b4k -- python3 bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k_prof.log 2>&1 || exit $?
S=$(find /tmp/b4k -name 'b4k_kernel_stats.csv' -print -quit)
cp "$S" gpurun_out/b4k_kernel_stats.csv
head -12 gpurun_out/b4k_kernel_stats.csv | cut -c1-160
