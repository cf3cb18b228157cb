# A/B of library build variants (pkc/libpkc<suffix>.so, selected through PKC_LIB) on the C2 bench.
# Usage: bash scripts/gpu_libab.sh "" _op4 _op16
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc$v.so timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-seq-configs --no-batch-sweep > gpurun_out/ab$v.log 2>&1 || exit $?
  echo "variant[$v] $(tail -1 gpurun_out/ab$v.log | cut -c1-170)"
done
