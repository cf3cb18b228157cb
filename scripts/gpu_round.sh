# Round evidence: GPU tests + smoke + bench (gpu_check.sh), bench under rocprofv3 + timeline,
# PMC traffic passes, then the sequence-model profile with and without the block-sparse W.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh || exit $?
grep -q '"metric"' gpurun_out/bench.log || exit 1
bash scripts/gpu_bench_prof.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
PKC_W_SPARSE=off timeout -k 10 300 python3 scripts/bench_seq.py --configs c3 --steps 20 > gpurun_out/seq_c3_wdense.log 2>&1 || exit $?
tail -2 gpurun_out/seq_c3_wdense.log
bash scripts/gpu_prof_seq.sh --steps 10 || exit $?
