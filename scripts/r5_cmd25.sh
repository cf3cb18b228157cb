set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
bash scripts/gpu.sh tests smoke bench || exit $?
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c4 --prec bf16 > gpurun_out/r5prof/trace_c4_bf16.json 2> gpurun_out/r5prof/trace_c4_bf16.err
echo "trace c4 rc=$?"; cat gpurun_out/r5prof/trace_c4_bf16.json | tr -d '\n' | cut -c1-1200; echo
