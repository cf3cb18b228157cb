set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_step.py tests/test_gpu_plugin.py tests/test_gpu_mlp.py tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_rnn.py tests/test_gpu_seq_graph.py tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r5_t2.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r5_t2.log | tail -25
PKC_ARGS="--configs c3,c4,c5 --steps 8 --warmup 2" timeout -k 10 900 bash scripts/gpu.sh treeab && cp gpurun_out/treeab.txt gpurun_out/r5_treeab_fp32.txt
PKC_ARGS="--configs c3,c4,c5 --steps 8 --warmup 2 --prec bf16" timeout -k 10 900 bash scripts/gpu.sh treeab && cp gpurun_out/treeab.txt gpurun_out/r5_treeab_bf16.txt
