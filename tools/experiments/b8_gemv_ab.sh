# 8-row decode: sgemv (default for 3-16 rows) vs the row-set GEMV (gemv.hip, M <= 8) for every projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/b8gemv; mkdir -p $O
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b8_default 300 "" --batch 8 --steps 6 --warmup 1
run b8_gemv 300 K8S_GEMV_MAX_M=8 --batch 8 --steps 6 --warmup 1
run b4_default 300 "" --batch 4 --steps 6 --warmup 1
run b4_gemv 300 K8S_GEMV_MAX_M=4 --batch 4 --steps 6 --warmup 1
