# Transposed-read staging of bf16 m-contiguous operands: GEMM parity tests, large-M TF/s, the
# B=4096 step and its kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out /tmp/b4k
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm" > gpurun_out/pytest_tr.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/pytest_tr.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_tr.log 2>&1 || exit $?
grep mlp gpurun_out/gemm_tr.log
timeout -k 10 300 python bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b4k.log').read().strip().splitlines()[-1]); print('B4096', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b4k -o b4k -- python3 bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k_prof.log 2>&1 || exit $?
S=$(find /tmp/b4k -name 'b4k_kernel_stats.csv' -print -quit)
cp "$S" gpurun_out/b4k_kernel_stats.csv
T=$(find /tmp/b4k -name 'b4k_kernel_trace.csv' -print -quit)
python3 scripts/trace_gaps.py "$T" > gpurun_out/b4k_timeline.txt
head -12 gpurun_out/b4k_kernel_stats.csv | cut -c1-160
tail -40 gpurun_out/b4k_timeline.txt
