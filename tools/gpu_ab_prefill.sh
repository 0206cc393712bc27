# TP=1 prefill A/B: hand-written GEMM routing (default) vs the library oracle, a TP=1 kernel table, and the
# recovery test.  Each GPU step has its own time limit; a timeout / abort / fault ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab; mkdir -p $O
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$O/$log"; exit $rc; fi
  return 0
}
step 300 bench_auto.json python -u bench.py --steps 6 --warmup 2
grep metric $O/bench_auto.json
K8S_GEMM=library step 300 bench_lib.json python -u bench.py --steps 6 --warmup 2
grep metric $O/bench_lib.json
step 400 test_multigpu.log python -u -m pytest tests/test_multigpu.py -x -v -s --timeout 380 --timeout-method thread
grep -E "passed|failed" $O/test_multigpu.log | tail -1
step 300 test_recovery_gpu.log python -u -m pytest tests/test_recovery_gpu.py -x -v -s --timeout 200 --timeout-method thread
grep -E "passed|failed" $O/test_recovery_gpu.log | tail -1
bash tools/gpu_prof.sh tp1_default "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -40 gpurun_out/rocprof_70b_tp1_default_kernels.txt
