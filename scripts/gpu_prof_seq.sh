# rocprofv3 kernel-trace + stats of the sequence-model bench: the stats summary comes back under
# gpurun_out/prof_seq/ (the raw trace stays in /tmp on the box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_seq /tmp/prof_seq
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_seq -o run -- python3 scripts/bench_seq.py "$@" > gpurun_out/prof_seq.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 1500 gpurun_out/prof_seq.log
[ $rc -eq 0 ] || exit $rc
f=$(find /tmp/prof_seq -name "*kernel_stats.csv" -print -quit)
cp "$f" gpurun_out/prof_seq/kernel_stats.csv
head -30 gpurun_out/prof_seq/kernel_stats.csv | cut -c1-220
