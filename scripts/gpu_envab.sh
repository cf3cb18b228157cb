# A/B of environment settings on the C2 bench: each argument is "VAR=value" (or "-" for none).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-seq-configs --no-batch-sweep > gpurun_out/env$i.log 2>&1 || exit $?
  else
    env "$v" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-seq-configs --no-batch-sweep > gpurun_out/env$i.log 2>&1 || exit $?
  fi
  echo "[$v] $(tail -1 gpurun_out/env$i.log | cut -c60-140)"
done
