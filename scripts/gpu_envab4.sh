# split-K budgets re-measured with the 8-column BatchNorm kernels (same box, two alternating rounds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/ab4_$name.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab4_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
run def PKC_X=0
run sf8 PKC_MAX_SPLITS_FWD=8
run sf6 PKC_MAX_SPLITS_FWD=6
run s6 PKC_MAX_SPLITS=6
run s8 PKC_MAX_SPLITS=8
done
