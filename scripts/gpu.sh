# One runner for every GPU-box recipe (run through gpurun from the repo root):
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh <recipe> [<recipe> ...]
#
# Recipes run in order; the first failing one ends the call (no GPU step after a fault, abort
# or time limit).  Every GPU step carries its own `timeout -k 10`.  Outputs land in gpurun_out/.
#
#   tests       pytest -m gpu (all GPU parity tests)          -> gpurun_out/pytest_gpu.log
#   smoke       __graft_entry__.smoke()                       -> gpurun_out/smoke.log
#   bench       python bench.py (the driver's default line)   -> gpurun_out/bench.log
#   bench_prof  the bench under rocprofv3 --kernel-trace --stats + the step timeline
#                                                             -> gpurun_out/bprof/
#   pmc         HBM traffic of the dominant launch: FETCH_SIZE and WRITE_SIZE passes
#               (PMC_PREC=fp32 PMC_OUT=pmc_traffic_fp32.json for the fp32 entry)
#                                                             -> gpurun_out/pmc_traffic*.json
#   mfma        MFMA counters of the C2 step (B=128, B=4096) and the C3/C4/C5 steps -> gpurun_out/mfma/
#   seq         scripts/bench_seq.py (C3/C4/C5/GRU)           -> gpurun_out/seq.log
#   seq_prof    bench_seq under rocprofv3 --kernel-trace --stats -> gpurun_out/prof_seq/
#   b4k_prof    the B=4096 step under rocprofv3 + timeline     -> gpurun_out/b4k/
#   dp2         bench.py --gpus 2 on one GPU over gloo (C2)    -> gpurun_out/dp2.log
#   seq_dp2     bench.py --gpus 2 --config c4 / c5 on one GPU over gloo -> gpurun_out/seq_dp2.log
#   kprof       scripts/kbench.py plain and under rocprofv3    -> gpurun_out/kprof/
#   ab          same-run A/B of one environment knob: AB_VAR over AB_VALUES (space-separated), two
#               alternating rounds of `python AB_CMD` (e.g. "bench.py --batch 4096 ...")
#                                                             -> gpurun_out/ab.txt
#   some        pytest of the files / node ids in PYTEST_SEL (space-separated) -> gpurun_out/pytest_some.log
#   treeab      same-box A/B of this tree against the tree in AB_TREE (a built worktree, default
#               _bis_r4): scripts/bench_seq.py $PKC_ARGS in each, two alternating rounds
#                                                             -> gpurun_out/treeab.txt
#   seq2        scripts/bench_seq.py in fp32 and in bf16 mode   -> gpurun_out/seq_fp32.log, seq_bf16.log
#   seq_prof2   bench_seq under rocprofv3 in fp32 and bf16 mode -> gpurun_out/prof_seq/{fp32,bf16}_kernel_stats.csv
#   trace       phase trace of the step kernels / persistent loops (libpkc_trace.so, built with
#               `python pytorch-kaldi-cgs_amd/pkc/_build.py --trace`): scripts/trace_steps.py
#               $TRACE_ARGS (e.g. "--config c3 --prec bf16 --persist") -> gpurun_out/trace.json
#   b_sweep     bench.py at B = 1024 / 4096 in fp32, bf16x3 and bf16   -> gpurun_out/b_sweep.txt
#   round       tests smoke bench bench_prof pmc
#
# Extra arguments for a recipe's python command: PKC_ARGS="..." (bench, seq, kprof).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
A=${PKC_ARGS:-}

ok() {   # exit status of the last step; stop the call on anything but 0
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  [ "$rc" -eq 0 ] || exit "$rc"
}

r_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?
  grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/pytest_gpu.log | tail -15
  ok $rc tests
}

r_some() {
  timeout -k 10 900 python -u -m pytest $PYTEST_SEL -m gpu -v -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_some.log 2>&1
  local rc=$?
  grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/pytest_some.log | tail -15
  ok $rc some
}

r_treeab() {
  local other=${AB_TREE:-_bis_r4}
  : > gpurun_out/treeab.txt
  for i in 1 2; do for t in . "$other"; do
    (cd "$t" && timeout -k 10 300 python -u scripts/bench_seq.py $A) > gpurun_out/treeab_run.log 2>&1
    ok $? "treeab $t"
    grep -E '^\{' gpurun_out/treeab_run.log | sed "s|^|tree=$t  |" | cut -c1-600 >> gpurun_out/treeab.txt
  done; done
  cat gpurun_out/treeab.txt
}

r_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  local rc=$?; tail -3 gpurun_out/smoke.log; ok $rc smoke
}

r_bench() {
  timeout -k 10 600 python -u bench.py $A > gpurun_out/bench.log 2>&1
  local rc=$?; tail -c 3000 gpurun_out/bench.log; ok $rc bench
}

r_bench_prof() {
  mkdir -p gpurun_out/bprof /tmp/bprof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bprof -o bench \
    -- python3 bench.py --no-cpu-baseline --no-batch-sweep > gpurun_out/bprof/bench.log 2>&1
  ok $? bench_prof
  local T S
  T=$(find /tmp/bprof -name 'bench_kernel_trace.csv' -print -quit)
  S=$(find /tmp/bprof -name 'bench_kernel_stats.csv' -print -quit)
  cp "$S" gpurun_out/bprof/bench_kernel_stats.csv
  gzip -c "$T" > gpurun_out/bprof/bench_kernel_trace.csv.gz
  # anchor: the heads' NLL launch (once per step; with the deferred tail the gather rides in a
  # grouped launch inside the multi-step graphs): the listing starts there, one whole step long
  # (steps holding a standalone batch_gather_kernel are single-step graph replays, not the timed
  # multi-step graphs: excluded)
  local NL
  NL=$(python3 -c "import json,sys; print(round(next(json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric')).get('graph_launches_per_step') or 25))" gpurun_out/bprof/bench.log)
  python3 scripts/trace_gaps.py "$T" nll_multi_kernel "<1, true" batch_gather_kernel "$NL" > gpurun_out/bprof/timeline.txt
  tail -3 gpurun_out/bprof/timeline.txt
}

r_pmc() {
  mkdir -p gpurun_out/pmc
  local N=20 K=${PMC_KERNEL:-pkc_gemm_grouped} P=${PMC_PREC:-bf16}
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o f \
    -- python3 bench.py --pmc-replay $N --pmc-kernel $K --prec $P > gpurun_out/pmc/fetch.log 2>&1
  ok $? pmc_fetch
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o w \
    -- python3 bench.py --pmc-replay $N --pmc-kernel $K --prec $P > gpurun_out/pmc/write.log 2>&1
  ok $? pmc_write
  python3 scripts/pmc_summary.py gpurun_out/pmc $N > gpurun_out/${PMC_OUT:-pmc_traffic.json}
  cat gpurun_out/${PMC_OUT:-pmc_traffic.json}
  rm -rf gpurun_out/pmc/fetch gpurun_out/pmc/write
}

r_mfma() {
  mkdir -p gpurun_out/mfma
  local C="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfma128 -o p -- python3 bench.py \
    --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/mfma/b128.log 2>&1
  ok $? mfma_b128
  python3 scripts/mfma_summary.py /tmp/mfma128 > gpurun_out/mfma/b128.json
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfma4k -o p -- python3 bench.py \
    --batch 4096 --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/mfma/b4096.log 2>&1
  ok $? mfma_b4096
  python3 scripts/mfma_summary.py /tmp/mfma4k > gpurun_out/mfma/b4096.json
  for c in c3 c4 c5; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfma$c -o p -- python3 scripts/bench_seq.py \
      --configs $c --steps 2 --warmup 1 > gpurun_out/mfma/$c.log 2>&1
    ok $? mfma_$c
    python3 scripts/mfma_summary.py /tmp/mfma$c > gpurun_out/mfma/$c.json
  done
  # the sequence configs' bf16 performance mode (bf16 projections and step products)
  for c in c3 c4 c5; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d /tmp/mfmab$c -o p -- python3 scripts/bench_seq.py \
      --configs $c --steps 2 --warmup 1 --prec bf16 > gpurun_out/mfma/${c}_bf16.log 2>&1
    ok $? mfma_${c}_bf16
    python3 scripts/mfma_summary.py /tmp/mfmab$c > gpurun_out/mfma/${c}_bf16.json
  done
  head -c 1500 gpurun_out/mfma/b4096.json
}

r_seq() {
  timeout -k 10 600 python -u scripts/bench_seq.py $A > gpurun_out/seq.log 2>&1
  local rc=$?; cat gpurun_out/seq.log | cut -c1-400; ok $rc seq
}

r_seq_prof() {
  mkdir -p gpurun_out/prof_seq /tmp/prof_seq
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_seq -o run \
    -- python3 scripts/bench_seq.py --steps 10 $A > gpurun_out/prof_seq.log 2>&1
  ok $? seq_prof
  cp "$(find /tmp/prof_seq -name '*kernel_stats.csv' -print -quit)" gpurun_out/prof_seq/kernel_stats.csv
  head -20 gpurun_out/prof_seq/kernel_stats.csv | cut -c1-200
}

r_b4k_prof() {
  mkdir -p gpurun_out/b4k /tmp/b4k
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b4k -o b4k -- python3 bench.py \
    --batch 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b4k/prof.log 2>&1
  ok $? b4k_prof
  cp "$(find /tmp/b4k -name 'b4k_kernel_stats.csv' -print -quit)" gpurun_out/b4k/kernel_stats.csv
  python3 scripts/trace_gaps.py "$(find /tmp/b4k -name 'b4k_kernel_trace.csv' -print -quit)" batch_gather \
    "<1, true" > gpurun_out/b4k/timeline.txt
  tail -5 gpurun_out/b4k/timeline.txt
}

r_dp2() {
  PKC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline \
    --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/dp2.log 2>&1
  local rc=$?; grep '^{' gpurun_out/dp2.log | cut -c1-400; ok $rc dp2
}

r_seq_dp2() {
  : > gpurun_out/seq_dp2.log
  for c in c4 c5; do
    PKC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config $c --steps 6 --warmup 2 \
      --no-cpu-baseline >> gpurun_out/seq_dp2.log 2>&1
    ok $? seq_dp2_$c
  done
  grep '^{' gpurun_out/seq_dp2.log | cut -c1-500
}

r_kprof() {
  mkdir -p gpurun_out/kprof
  timeout -k 10 300 python scripts/kbench.py $A > gpurun_out/kbench.log 2>&1
  ok $? kbench
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o k \
    -- python3 scripts/kbench.py $A > gpurun_out/kprof.log 2>&1
  ok $? kprof
}

r_ab() {
  : > gpurun_out/ab.txt
  for i in 1 2; do for v in $AB_VALUES; do
    env "$AB_VAR=$v" timeout -k 10 300 python -u $AB_CMD > gpurun_out/ab_run.log 2>&1
    ok $? "ab $AB_VAR=$v"
    grep -E '^\{|^ *[a-z0-9].*(TF/s|us)' gpurun_out/ab_run.log | sed "s|^|$AB_VAR=$v  |" | cut -c1-400 >> gpurun_out/ab.txt
  done; done
  cat gpurun_out/ab.txt
}

r_seq2() {
  for P in fp32 bf16; do
    timeout -k 10 600 python -u scripts/bench_seq.py --prec $P $A > gpurun_out/seq_$P.log 2>&1
    ok $? seq_$P
    grep '^{' gpurun_out/seq_$P.log | cut -c1-400
  done
}

r_seq_prof2() {
  mkdir -p gpurun_out/prof_seq
  for P in fp32 bf16; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pseq$P -o run \
      -- python3 scripts/bench_seq.py --steps 6 --warmup 2 --prec $P $A > gpurun_out/prof_seq/$P.log 2>&1
    ok $? seq_prof_$P
    cp "$(find /tmp/pseq$P -name '*kernel_stats.csv' -print -quit)" gpurun_out/prof_seq/${P}_kernel_stats.csv
    head -8 gpurun_out/prof_seq/${P}_kernel_stats.csv | cut -c1-160
  done
}

r_trace() {
  PKC_LIB=$GRAFT_REPO_ROOT/pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so timeout -k 10 300 \
    python -u scripts/trace_steps.py ${TRACE_ARGS:-} > gpurun_out/trace.json 2> gpurun_out/trace.err
  ok $? trace
  tr -d '\n' < gpurun_out/trace.json | cut -c1-1200; echo
}

r_b_sweep() {
  : > gpurun_out/b_sweep.txt
  for P in fp32 bf16x3 bf16; do for B in 1024 4096; do
    timeout -k 10 300 python -u bench.py --batch $B --prec $P --steps 150 --warmup 10 --no-cpu-baseline \
      --no-batch-sweep --no-fp32 --no-seq-configs > gpurun_out/b_run.log 2>&1
    ok $? "bench B=$B $P"
    grep '^{' gpurun_out/b_run.log | cut -c1-160 | sed "s|^|B=$B $P  |" >> gpurun_out/b_sweep.txt
  done; done
  cat gpurun_out/b_sweep.txt
}

[ $# -gt 0 ] || { sed -n 2,30p "$0"; exit 2; }
for r in "$@"; do
  if [ "$r" = round ]; then
    set -- tests smoke bench bench_prof pmc
    for q in "$@"; do "r_$q"; done
  else
    "r_$r"
  fi
done
