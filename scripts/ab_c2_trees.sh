# Same-box A/B of the C2 headline step (bench.py, B = 128, bf16 products) between this tree and a
# built worktree (AB_TREE, default _bis_r5): three alternating rounds, one JSON summary per run.
#
#   gpurun --timeout 1200 -- 'bash scripts/ab_c2_trees.sh'          -> gpurun_out/c2ab.txt
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
other=${AB_TREE:-_bis_r5}
: > gpurun_out/c2ab.txt
for i in 1 2 3; do for t in . "$other"; do
  (cd "$t" && timeout -k 10 300 python -u bench.py --steps 400 --warmup 40 --no-cpu-baseline \
    --no-batch-sweep --no-fp32 --no-seq-configs) > gpurun_out/c2ab_run.log 2>&1
  rc=$?
  echo "[c2ab $t] rc=$rc"
  [ "$rc" -eq 0 ] || exit "$rc"
  grep -E '^\{' gpurun_out/c2ab_run.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('tree=$t', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['step_breakdown_us'].get('dense_fwd N=1024'), d['step_breakdown_us'].get('dense_bwd N=1024'))
" >> gpurun_out/c2ab.txt
done; done
cat gpurun_out/c2ab.txt
