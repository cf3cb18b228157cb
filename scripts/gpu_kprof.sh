# kernel micro-benchmarks, plain and under rocprofv3 kernel-trace (pure kernel durations)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kprof
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kbench.py "$@" > gpurun_out/kbench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o k -- python3 scripts/kbench.py "$@" > gpurun_out/kprof.log 2>&1
echo "rc=$?"
