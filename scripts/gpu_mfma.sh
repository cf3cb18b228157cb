# MFMA utilisation (rocprofv3 --pmc: MFMA MOPS, MFMA busy cycles, GRBM_GUI_ACTIVE) of the C2 step at
# B = 128 (headline) and B = 4096 (batch sweep), and of the C4 sequence step; one pass each
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mfma
export TMPDIR=/tmp
C="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfma128 -o p -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/mfma/b128.log 2>&1 || exit $?
python3 scripts/mfma_summary.py /tmp/mfma128 > gpurun_out/mfma/b128.json && cat gpurun_out/mfma/b128.json
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfma4k -o p -- python3 bench.py --batch 4096 --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/mfma/b4096.log 2>&1 || exit $?
python3 scripts/mfma_summary.py /tmp/mfma4k > gpurun_out/mfma/b4096.json && cat gpurun_out/mfma/b4096.json
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfmac4 -o p -- python3 scripts/bench_seq.py --configs c4 --steps 2 --warmup 1 > gpurun_out/mfma/c4.log 2>&1 || exit $?
python3 scripts/mfma_summary.py /tmp/mfmac4 > gpurun_out/mfma/c4.json && cat gpurun_out/mfma/c4.json
