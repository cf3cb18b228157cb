set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in _bis_1aa71b4 _bis_14ccfaa .; do
  for i in 1 2; do
    (cd $t && timeout -k 10 200 python bench.py --no-cpu-baseline --no-batch-sweep $( [ $t = _bis_1aa71b4 ] || echo --no-fp32 ) --no-seq-configs > /tmp/hb.log 2>&1) || { tail -20 /tmp/hb.log; exit 1; }
    python -c "import json; d=json.loads(open('/tmp/hb.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'])"
  done
done
