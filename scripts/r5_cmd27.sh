set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
: > gpurun_out/r5prof/x3ab.txt
for i in 1 2; do for v in 1 0; do
PKC_X3_GROUPED_BIG=$v timeout -k 10 300 python -u bench.py --batch $B --prec bf16x3 --steps 60 --warmup 10 --no-cpu-baseline --no-batch-sweep --no-seq-configs --no-fp32 > gpurun_out/r5prof/x3_run.log 2>&1
rc=$?; echo "B=$B x3_grouped_big=$v rc=$rc $(grep '^{' gpurun_out/r5prof/x3_run.log | cut -c1-110)" | tee -a gpurun_out/r5prof/x3ab.txt
[ $rc -eq 0 ] || exit $rc
done; done
