# recovery + replica GPU tests (verbose, own time limits), then the big-tile GEMM tuning sweep (--write).
# A test that FAILS (rc 1) does not stop the sweep; a timeout, abort or fault (any other rc) ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 "gpurun_out/$log"; exit $rc; fi
  return 0
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step 170 recov.log python -u -m pytest tests/test_recovery_gpu.py -x -v -s --timeout 160 --timeout-method thread
  step 170 repl.log python -u -m pytest tests/test_replicas_gpu.py -x -v -s --timeout 160 --timeout-method thread
fi
step ${TUNE_TIMEOUT:-900} pgemm_tune.txt python -u tools/pgemm_tune.py ${TUNE_ARGS:---tp 1 2 4 8 --m 192 256 384 512 768 1024 2048 4096 8192 --only qkv o_proj gate_up down} --json-out gpurun_out/pgemm_tune.json --write
cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json gpurun_out/pgemm_gfx950.json
tail -5 gpurun_out/pgemm_tune.txt
