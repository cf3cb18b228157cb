set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_mlp.py tests/test_gpu_seq.py tests/test_gpu_kernels.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r5_t3.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r5_t3.log | tail -25
mkdir -p gpurun_out/r5prof
for P in fp32 bf16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseq$P -o run \
    -- python3 scripts/bench_seq.py --configs c3,c4,c5 --steps 6 --warmup 2 --prec $P > gpurun_out/r5prof/seq_$P.log 2>&1
  echo "seq_prof $P rc=$?"
  cp "$(find /tmp/pseq$P -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5prof/seq_${P}_kernel_stats.csv
done
C="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfmac4b -o p -- python3 scripts/bench_seq.py \
      --configs c4 --steps 2 --warmup 1 --prec bf16 > gpurun_out/r5prof/mfma_c4_bf16.log 2>&1 && python3 scripts/mfma_summary.py /tmp/mfmac4b 12 > gpurun_out/r5prof/mfma_c4_bf16.json
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfmac4 -o p -- python3 scripts/bench_seq.py \
      --configs c4 --steps 2 --warmup 1 > gpurun_out/r5prof/mfma_c4.log 2>&1 && python3 scripts/mfma_summary.py /tmp/mfmac4 12 > gpurun_out/r5prof/mfma_c4.json
C2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
timeout -s KILL 240 rocprofv3 --pmc $C2 --output-format csv -d /tmp/sqc5 -o p -- python3 scripts/bench_seq.py \
      --configs c5 --steps 2 --warmup 1 > gpurun_out/r5prof/sq_c5.log 2>&1; echo "sq c5 rc=$?"
cp "$(find /tmp/sqc5 -name '*counter_collection.csv' -print -quit)" gpurun_out/r5prof/sq_c5_counters.csv 2>/dev/null
for P in fp32 bf16x3 bf16; do for B in 1024 4096; do
  timeout -k 10 300 python -u bench.py --batch $B --prec $P --steps 150 --warmup 10 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/r5prof/b${B}_$P.log 2>&1
  echo "bench B=$B $P rc=$?"; grep '^{' gpurun_out/r5prof/b${B}_$P.log | cut -c1-160
done; done
timeout -k 5 60 ./scripts/mfma_layout_probe > gpurun_out/r5prof/mfma_layout_probe.txt 2>&1; echo "probe rc=$?"
ls -la gpurun_out/r5prof
