set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
bash scripts/gpu.sh tests || exit $?
grep -E "persist|bf16_vs_bf16" gpurun_out/pytest_gpu.log | head -5
for c in c3 c4; do
timeout -k 10 300 python -u scripts/bench_seq.py --configs $c --prec bf16 --steps 8 --warmup 2 > gpurun_out/r5prof/${c}b_fg.log 2>&1
echo "$c bf16 rc=$? $(grep '^{' gpurun_out/r5prof/${c}b_fg.log | cut -c150-260)"
done
