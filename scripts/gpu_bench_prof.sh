# The bench command itself under rocprofv3 --kernel-trace --stats (the summary the bench's
# roofline must agree with) + its step timeline; then the PMC traffic passes.  The raw trace
# stays in /tmp on the box (it is larger than what gpurun copies back); only the stats summary,
# the timeline and the bench line come back under gpurun_out/bprof.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bprof /tmp/bprof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bprof -o bench -- python3 bench.py --no-cpu-baseline --no-batch-sweep > gpurun_out/bprof/bench.log 2>&1 || exit $?
T=$(find /tmp/bprof -name 'bench_kernel_trace.csv' -print -quit)
S=$(find /tmp/bprof -name 'bench_kernel_stats.csv' -print -quit)
cp "$S" gpurun_out/bprof/bench_kernel_stats.csv
python3 scripts/trace_gaps.py "$T" batch_gather "gemm_grouped_kernel<1, true" > gpurun_out/bprof/timeline.txt
tail -3 gpurun_out/bprof/timeline.txt
