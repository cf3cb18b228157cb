# C2 launch knobs re-measured on bf16-stored operands (same box, two alternating rounds):
# default, PKC_GEMM_DEPTH=8, PKC_MAX_SPLITS_FWD=8, PKC_MAX_SPLITS=5, PKC_MAX_SPLITS=3
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bf16" > gpurun_out/pytest_ab2.log 2>&1 || { tail -20 gpurun_out/pytest_ab2.log; exit 1; }
PKC_GEMM_DEPTH=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab2_d8.log 2>&1 || { tail -20 gpurun_out/pytest_ab2_d8.log; exit 1; }
tail -1 gpurun_out/pytest_ab2_d8.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/ab2_$name.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab2_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
run def PKC_X=0
run d8 PKC_GEMM_DEPTH=8
run sf8 PKC_MAX_SPLITS_FWD=8
run s5 PKC_MAX_SPLITS=5
run s3 PKC_MAX_SPLITS=3
done
for v in 4 8; do
PKC_GEMM_DEPTH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/ab2_sweep$v.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/ab2_sweep$v.log').read().strip().splitlines()[-1]); print('depth $v sweep', d['batch_sweep_frames_per_s'])"
done
