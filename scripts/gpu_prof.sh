# rocprofv3 kernel-trace + stats of a short bench run (writes gpurun_out/prof/)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 1500 gpurun_out/prof_bench.log
