# A/B of the round-3 launch changes on the bench line (PKC_DEFER_TAIL: the first layer's update
# riding in the next step's gather launch; PKC_DENSE_XCD: the BatchNorm kernels' column groups on
# the XCD that produced their slabs), after their bit-identity / parity tests
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "graph_replay or dense_bn or c2_bf16 or c1_full" > gpurun_out/pt_defer.log 2>&1
rc=$?; tail -3 gpurun_out/pt_defer.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for cfg in "0 1" "1 1" "0 2" "1 2"; do set -- $cfg
PKC_DEFER_TAIL=$1 PKC_DENSE_XCD=$2 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-batch-sweep --no-seq-configs --no-fp32 > gpurun_out/ab_defer.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/ab_defer.log'):
    if l.startswith('{\"metric'): d=json.loads(l); print('defer=$1 xcd=$2', d['value'], d['ms_per_step'], d['launches_per_step'], d['roofline']['frac'])
"
done; done
