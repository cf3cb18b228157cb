# Round-end evidence in one call: GPU tests + smoke + the bench line (scripts/gpu_check.sh), the
# rocprofv3 kernel-trace/stats of the bench command and its step timeline
# (scripts/gpu_bench_prof.sh), then the PMC traffic passes of the dominant launch (scripts/gpu_pmc.sh).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh || exit $?
grep -q '"metric"' gpurun_out/bench.log || exit 1
bash scripts/gpu_bench_prof.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
