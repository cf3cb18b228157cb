# Recurrent-path parity tests, then the sequence-model bench for the given configs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFGS=${1:-c3,c4,c5,gru}
timeout -k 10 400 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_seq.py tests/test_gpu_quant_step.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/rnn.log 2>&1
rc=$?; tail -5 gpurun_out/rnn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_seq.py --configs "$CFGS" > gpurun_out/seq.log 2>&1
rc=$?; tail -4 gpurun_out/seq.log; exit $rc
