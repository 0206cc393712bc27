# Round check on one MI355X: focused GPU tests, the fp8 big-tile GEMM sweep (merged into the plan table), the
# driver's default bench and its rocprof kernel table.  Test failures (rc 1) do not stop later steps; a timeout,
# abort or fault (any other rc) ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/round; mkdir -p $O
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$O/$log"; exit $rc; fi
  return 0
}
if [ -z "${SKIP_TESTS:-}" ]; then
  for t in ${TESTS:-test_recovery_gpu test_replicas_gpu test_xgmi_gpu test_multigpu test_model_gpu test_pgemm_gpu}; do
    step 330 $t.log python -u -m pytest tests/$t.py -x -v -s --timeout 320 --timeout-method thread
    grep -E "passed|failed" $O/$t.log | tail -1
  done
fi
if [ -n "${TUNE_FP8:-}" ]; then
  step 600 tune_fp8.txt python -u tools/pgemm_tune.py --fp8 --tp 1 2 4 8 --m 192 256 384 512 768 1024 2048 4096 8192 --only qkv o_proj gate_up down --json-out $O/tune_fp8.json --write
  tail -3 $O/tune_fp8.txt
  cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950.json
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  step 600 bench_default.json python -u bench.py --gpus 1 --steps ${BENCH_STEPS:-10} --warmup 3
  cat $O/bench_default.json
  bash tools/gpu_prof.sh tp1_default "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  head -24 gpurun_out/rocprof_70b_tp1_default_kernels.txt
fi
