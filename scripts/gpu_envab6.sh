# optimizer spread and XCD remap re-measured on the bf16 / 8-column-BN step (same box, two alternating rounds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/ab6_$name.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab6_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
run def PKC_X=0
run sp300 PKC_OPT_SPREAD_PARAMS=300000
run sp700 PKC_OPT_SPREAD_PARAMS=700000
run sp1m PKC_OPT_SPREAD_PARAMS=1000000
run xcd0 PKC_GEMM_XCD=0
done
