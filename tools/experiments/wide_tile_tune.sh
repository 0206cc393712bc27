# (Round-5 probe; the 64 x 256 tiles it tuned, configs 37 / 38, were removed again: no gain -- profiles/mgemm_wide_tile_tune_r5.txt.)
# Re-tune the mgemm plans after adding the 64 x 256 tiles (configs 37 / 38): bf16 (TP = 1 / 2 / 4 / 8) and the fp8
# MX modes (TP = 1 / 4) at 32-128 rows, then the batch-64 / 32 A/B rows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/wide; mkdir -p $O
timeout -k 10 600 python -u tools/mgemm_tune.py --tp 1 2 4 8 --m 32 64 128 --only qkv o_proj gate_up down --write > $O/tune_bf16.txt 2>&1 || { tail -20 $O/tune_bf16.txt; exit 1; }
timeout -k 10 400 python -u tools/mgemm_tune.py --mx --tp 1 4 --m 32 64 128 --write > $O/tune_mx.txt 2>&1 || { tail -20 $O/tune_mx.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/mgemm_gfx950.json
grep -v cand $O/tune_bf16.txt | tail -50
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b64 600 --batch 64 --steps 3 --warmup 1
run b32 600 --batch 32 --steps 3 --warmup 1
run tp8_b64 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run fp8_b64 600 --dtype fp8 --batch 64 --steps 3 --warmup 1
