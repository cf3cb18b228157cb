# rocprofv3 kernel-trace + stats of the sequence-model bench (writes gpurun_out/prof_seq/)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_seq
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seq -o run -- python3 scripts/bench_seq.py "$@" > gpurun_out/prof_seq.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 1500 gpurun_out/prof_seq.log
f=$(find gpurun_out/prof_seq -name "*kernel_stats.csv" | head -1); echo "$f"; head -30 "$f" | cut -c1-220
