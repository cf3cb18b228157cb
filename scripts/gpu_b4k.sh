# Large-batch step: split-K dW + slab sums, parallel BatchNorm finalize.  Parity tests (MLP engine,
# kernels, DP, sequence configs that share the BN kernels), then B = 1024 / 4096 / 128 steps and the
# B = 4096 kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out /tmp/b4k
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py tests/test_gpu_dp.py tests/test_gpu_seq.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_b4k.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_b4k.log
[ $rc -eq 0 ] || exit $rc
for b in 4096 1024; do
timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b$b.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b$b.log').read().strip().splitlines()[-1]); print('B$b', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b128.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b128.log').read().strip().splitlines()[-1]); print('B128', d['value'], d['ms_per_step'])"
timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4 --steps 10 > gpurun_out/seq_b4k.log 2>&1 || exit $?
grep '^{' gpurun_out/seq_b4k.log | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b4k -o b4k -- python3 bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k_prof.log 2>&1 || exit $?
S=$(find /tmp/b4k -name 'b4k_kernel_stats.csv' -print -quit)
cp "$S" gpurun_out/b4k_kernel_stats.csv
T=$(find /tmp/b4k -name 'b4k_kernel_trace.csv' -print -quit)
python3 scripts/trace_gaps.py "$T" > gpurun_out/b4k_timeline.txt
tail -48 gpurun_out/b4k_timeline.txt
