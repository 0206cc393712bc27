# bf16 17-64-row decode: which pre-norm projections take mgemm's RMS prologue (sums of squares on the MFMA from
# 8192 features) and which a separate RMSNorm + plain GEMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rmspol; mkdir -p $O
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
for rep in 1; do
run b64_qkvsep_gufused_$rep 600 "" --batch 64 --steps 3 --warmup 1
run b64_allfused_$rep 600 K8S_RMS_UNFUSED_MAX_M=0 --batch 64 --steps 3 --warmup 1
run b64_allsep_$rep 600 K8S_RMS_PROLOGUE_SWIGLU=0 --batch 64 --steps 3 --warmup 1
done
run b32_qkvsep_gufused 600 "" --batch 32 --steps 3 --warmup 1
run b32_allfused 600 K8S_RMS_UNFUSED_MAX_M=0 --batch 32 --steps 3 --warmup 1
run b32_allsep 600 K8S_RMS_PROLOGUE_SWIGLU=0 --batch 32 --steps 3 --warmup 1
