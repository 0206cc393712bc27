# bf16 17-128-row plans tuned in situ (O / down with the residual epilogue, gate/up with the RMS prologue): the
# batch-64 / 32 rows with the shipped table, then the re-tune, then the same rows with the new table (one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/insitu; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b64_old 600 --batch 64 --steps 3 --warmup 1
run b32_old 600 --batch 32 --steps 3 --warmup 1
run tp8_b64_old 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --tp 1 8 --m 32 64 --only qkv o_proj gate_up down --write > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/mgemm_gfx950.json
grep -v cand $O/tune.txt | tail -20
run b64_new 600 --batch 64 --steps 3 --warmup 1
run b32_new 600 --batch 32 --steps 3 --warmup 1
run tp8_b64_new 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
