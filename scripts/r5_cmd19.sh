set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5prof; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_seq.py -k "persist or ligru_hcgs" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_t20.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|T <= " gpurun_out/r5_t20.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_seq.py --configs c3 --prec bf16 --steps 8 --warmup 2 > gpurun_out/r5prof/c3b_la.log 2>&1
echo "c3 bf16 (balanced plans) rc=$? $(grep '^{' gpurun_out/r5prof/c3b_la.log | cut -c1-250)"
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c3 --prec bf16 --persist > gpurun_out/r5prof/trace_c3_persist_la.json 2> gpurun_out/r5prof/trace_c3_persist_la.err
echo "trace rc=$?"; python3 -c "
import json; d=json.load(open('gpurun_out/r5prof/trace_c3_persist_la.json'))
for k in ('forward loop','BPTT loop'): print(k, d[k]['T'], d[k]['cycles_per_step_wave_mean'])
"
PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 python -u scripts/trace_steps.py --config c5 > gpurun_out/r5prof/trace_c5_qx2b.json 2> gpurun_out/r5prof/trace_c5_qx2b.err
echo "trace c5 rc=$?"; cat gpurun_out/r5prof/trace_c5_qx2b.json | tr -d '\n' | cut -c1-900; echo
