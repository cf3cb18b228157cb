# The bench command itself under rocprofv3 --kernel-trace --stats (the summary the bench's
# roofline must agree with) + its step timeline; then the PMC traffic passes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bprof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bprof -o bench -- python3 bench.py --no-cpu-baseline --no-batch-sweep > gpurun_out/bprof/bench.log 2>&1 || exit $?
python3 scripts/trace_gaps.py gpurun_out/bprof/bench_kernel_trace.csv > gpurun_out/bprof/timeline.txt
tail -3 gpurun_out/bprof/timeline.txt
