set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_seq.py tests/test_gpu_seq_graph.py tests/test_gpu_configs.py -k "persist or ligru or bf16 or c3" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t23.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|T <= " gpurun_out/r5_t23.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u scripts/bench_seq.py --configs c3 --prec bf16 --steps 8 --warmup 2 > gpurun_out/r5prof/c3b_pair.log 2>&1
echo "c3 bf16 rc=$? $(grep '^{' gpurun_out/r5prof/c3b_pair.log | cut -c150-260)"
done
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c3 --prec bf16 --persist > gpurun_out/r5prof/trace_c3_persist_pair.json 2> gpurun_out/r5prof/trace_c3_persist_pair.err
echo "trace rc=$?"; python3 -c "
import json; d=json.load(open('gpurun_out/r5prof/trace_c3_persist_pair.json'))
for k in ('forward loop','BPTT loop'): print(k, d[k]['T'], d[k]['cycles_per_step_wave_mean'])
"
