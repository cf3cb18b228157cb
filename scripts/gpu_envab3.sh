# k-tiles in flight for bf16-stored operands: standalone (PKC_GEMM_DEPTH) vs grouped
# (PKC_GEMM_DEPTH_G) launches, C2 step and batch sweep, two alternating rounds (same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PKC_GEMM_DEPTH=8 PKC_GEMM_DEPTH_G=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bf16" > gpurun_out/pytest_ab3.log 2>&1 || { tail -20 gpurun_out/pytest_ab3.log; exit 1; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs > gpurun_out/ab3_$name.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab3_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['batch_sweep_frames_per_s'])"
}
for r in 1 2; do
run def PKC_X=0
run d8s PKC_GEMM_DEPTH=8
run d8g PKC_GEMM_DEPTH_G=8
done
