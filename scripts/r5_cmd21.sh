set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_seq.py --configs c3 --prec bf16 --steps 8 --warmup 2 > gpurun_out/r5prof/c3b_x.log 2>&1
echo "c3 bf16 rc=$? $(grep '^{' gpurun_out/r5prof/c3b_x.log | cut -c150-260)"
