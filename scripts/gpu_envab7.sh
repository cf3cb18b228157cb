# optimizer spread threshold above 1M parameters (same box, two alternating rounds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-fp32 --no-seq-configs --no-batch-sweep > gpurun_out/ab7_$name.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab7_$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
run def PKC_X=0
run sp2500 PKC_OPT_SPREAD_PARAMS=2500000
run sp1500 PKC_OPT_SPREAD_PARAMS=1500000
run sp2500 PKC_OPT_SPREAD_PARAMS=2500000
run sp1200 PKC_OPT_SPREAD_PARAMS=1200000
done
