# C2 step: slab-budget knobs re-measured after the transposed-read staging (same run)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/bs.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'])" "$@"
}
run PKC_MAX_SPLITS=4
run PKC_MAX_SPLITS=6
run PKC_MAX_SPLITS=8
run PKC_MAX_SPLITS=4 PKC_MAX_SPLITS_FWD=8
run PKC_MAX_SPLITS=8 PKC_MAX_SPLITS_FWD=4
run PKC_MAX_SPLITS=4
