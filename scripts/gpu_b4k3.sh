# B = 4096 step kernel stats and timeline with bf16-stored operands (rocprofv3 kernel trace)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/b4k3 /tmp/b4k3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b4k3 -o b4k -- python3 bench.py --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k3/prof.log 2>&1 || exit $?
S=$(find /tmp/b4k3 -name 'b4k_kernel_stats.csv' -print -quit)
T=$(find /tmp/b4k3 -name 'b4k_kernel_trace.csv' -print -quit)
cp "$S" gpurun_out/b4k3/kernel_stats.csv
python3 scripts/trace_gaps.py "$T" batch_gather "gemm_grouped_kernel<1, true" > gpurun_out/b4k3/timeline.txt
cat gpurun_out/b4k3/timeline.txt
