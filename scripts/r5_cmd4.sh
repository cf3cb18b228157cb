set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -m gpu -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_persist.log 2>&1
rc=$?; echo "persist test rc=$rc"; grep -E "step [0-9]|passed|failed|Error" gpurun_out/r5_persist.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_mlp.py tests/test_gpu_seq.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_rnn.py tests/test_gpu_quant_step.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r5_t4.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r5_t4.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for P in bf16 fp32; do
  timeout -k 10 400 python -u scripts/bench_seq.py --configs c3,c4,c5 --steps 8 --warmup 2 --prec $P > gpurun_out/r5prof/seq_$P.log 2>&1
  echo "seq $P rc=$?"; grep '^{' gpurun_out/r5prof/seq_$P.log | cut -c1-330
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseqb -o run -- python3 scripts/bench_seq.py --configs c3,c4,c5 --steps 6 --warmup 2 --prec bf16 > gpurun_out/r5prof/seqprof_bf16.log 2>&1
echo "seq_prof bf16 rc=$?"; cp "$(find /tmp/pseqb -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/seq_bf16_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseqf -o run -- python3 scripts/bench_seq.py --configs c3,c4,c5 --steps 6 --warmup 2 > gpurun_out/r5prof/seqprof_fp32.log 2>&1
echo "seq_prof fp32 rc=$?"; cp "$(find /tmp/pseqf -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/seq_fp32_kernel_stats.csv
for P in fp32 bf16x3 bf16; do for B in 1024 4096; do
  timeout -k 10 300 python -u bench.py --batch $B --prec $P --steps 150 --warmup 10 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/r5prof/b${B}_$P.log 2>&1
  echo "bench B=$B $P rc=$?"; grep '^{' gpurun_out/r5prof/b${B}_$P.log | cut -c1-140
done; done
