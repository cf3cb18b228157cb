# All GPU tests, then A/B timings of the round's kernel changes:
#   sequence configs with PKC_RNN_BWD_GATES auto vs split, the C2 bench with PKC_FUSE_DW_OPT 1 vs 0.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_seq.py > gpurun_out/seq_auto.log 2>&1 || exit $?
PKC_RNN_BWD_GATES=split timeout -k 10 300 python scripts/bench_seq.py > gpurun_out/seq_split.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-seq-configs --no-batch-sweep > gpurun_out/bench_fused.log 2>&1 || exit $?
PKC_FUSE_DW_OPT=0 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-seq-configs --no-batch-sweep > gpurun_out/bench_nofuse.log 2>&1 || exit $?
grep -h '^{' gpurun_out/seq_auto.log gpurun_out/seq_split.log | cut -c1-150
tail -1 gpurun_out/bench_fused.log | cut -c1-200
tail -1 gpurun_out/bench_nofuse.log | cut -c1-200
