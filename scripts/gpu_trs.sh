# Transposed-read staging in the 64x64 body: GEMM + MLP parity tests, kbench gemm, the C2 step
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_trs.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_trs.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/kbench.py gemm > gpurun_out/kb_trs.log 2>&1 || exit $?
grep "bf16in" gpurun_out/kb_trs.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/btrs.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/btrs.log').read().strip().splitlines()[-1]); print('C2', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --batch 1024 --steps 50 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b1k.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b1k.log').read().strip().splitlines()[-1]); print('B1024', d['value'], d['ms_per_step'])"
