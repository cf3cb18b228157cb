# bench.py --gpus 2 rehearsal on one GPU (two ranks over gloo) with the bf16-stored operands
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PKC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/dp2.log 2>&1; rc=$?; echo "rc=$rc"
grep '^{' gpurun_out/dp2.log | cut -c1-300
tail -3 gpurun_out/dp2.log | cut -c1-200
exit $rc
