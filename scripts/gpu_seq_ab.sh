# Recurrent step kernels: parity tests, then the sequence configs' throughput; C2 step A/B of the
# one-shot forward GEMM (PKC_GEMM_1SHOT=0/1)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_quant_step.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seq.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_seq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4,c5 --steps 20 > gpurun_out/seq_ab.log 2>&1 || exit $?
grep '^{' gpurun_out/seq_ab.log | cut -c1-200
for v in 0 1 0 1; do
PKC_GEMM_1SHOT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b1shot$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b1shot$v.log').read().strip().splitlines()[-1]); print('1shot=$v', d['value'], d['ms_per_step'])"
done
