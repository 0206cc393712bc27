# 8-row decode: attention on the split kernel for up to 64 (sequence, kv head) pairs vs the one-workgroup kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/b8attn; mkdir -p $O
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b8_default 300 "" --batch 8 --steps 6 --warmup 1
run b8_split64 300 K8S_ATTN_SPLIT_PAIRS=64 --batch 8 --steps 6 --warmup 1
run b8_split128 300 K8S_ATTN_SPLIT_PAIRS=128 --batch 8 --steps 6 --warmup 1
run b8_default2 300 "" --batch 8 --steps 6 --warmup 1
