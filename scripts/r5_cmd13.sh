set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
for P in bf16x3 fp32; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb4k$P -o run -- python3 bench.py --batch 4096 --prec $P --steps 20 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-seq-configs --no-fp32 > gpurun_out/r5prof/b4k_$P.log 2>&1
echo "b4k $P rc=$? $(grep '^{' gpurun_out/r5prof/b4k_$P.log | cut -c1-120)"
cp "$(find /tmp/pb4k$P -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/b4k_${P}_kernel_stats.csv; head -12 gpurun_out/r5prof/b4k_${P}_kernel_stats.csv | cut -c1-200
done
