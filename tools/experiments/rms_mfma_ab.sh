# bf16 batched decode A/B of the RMS prologue on the MFMA (x . x^T diagonal) vs v_dot2 squares vs a separate RMSNorm
# launch (K8S_RMS_UNFUSED_MAX_M: rows up to which the >= 8192-feature projections take the separate norm).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rmsab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mgemm_gpu.py tests/test_model_gpu.py tests/test_mx_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b64_default 600 "" --batch 64 --steps 3 --warmup 1
run b64_unfused_r4 600 "K8S_RMS_UNFUSED_MAX_M=64 K8S_RMS_MFMA=0" --batch 64 --steps 3 --warmup 1
run tp8_b64_default 600 "" --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run b32_default 600 "" --batch 32 --steps 3 --warmup 1
