# Focused GPU test run: each file under its own time limit; a failing test (rc 1) does not stop the next file,
# a timeout / abort / fault ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for spec in ${FOCUS:-tests/test_recovery_gpu.py tests/test_replicas_gpu.py tests/test_model_gpu.py}; do
  log=gpurun_out/focus_$(basename "${spec%%::*}" .py).log
  timeout -k 10 ${FOCUS_TIMEOUT:-170} python -u -m pytest "$spec" -x -v -s --timeout 160 --timeout-method thread > "$log" 2>&1
  rc=$?
  echo "$spec rc=$rc"; grep -E "passed|failed" "$log" | tail -1
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$log"; exit $rc; fi
done
