# recurrent dW / dU split-K cap 4 (default) vs 8: sequence configs alternating (same box)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rc=0
echo "no tests in this A/B"
[ $rc -eq 0 ] || exit $rc
for v in 4 8 4 8; do
PKC_REC_DW_SPLITS=$v timeout -k 10 300 python scripts/bench_seq.py --configs c3,c4,c5,gru --steps 16 > gpurun_out/recsplit8_$v.log 2>&1 || exit $?
echo "splits=$v"; grep '^{' gpurun_out/recsplit8_$v.log | cut -c1-105
done
