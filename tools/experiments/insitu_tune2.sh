# The in-situ bf16 re-tune for the remaining row buckets / TP degrees (TP = 2 / 4 at 32-64 rows, TP = 1 / 8 at 128
# rows), with before / after rows on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/insitu2; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run tp4_b64_old 600 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run b96_old 600 --batch 96 --steps 2 --warmup 1
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --tp 2 4 --m 32 64 --only qkv o_proj gate_up down --write > $O/tune_a.txt 2>&1 || { tail -20 $O/tune_a.txt; exit 1; }
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --tp 1 8 --m 128 --only qkv o_proj gate_up down --write > $O/tune_b.txt 2>&1 || { tail -20 $O/tune_b.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/mgemm_gfx950.json
cat $O/tune_a.txt $O/tune_b.txt | grep -v cand | tail -30
run tp4_b64_new 600 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run b96_new 600 --batch 96 --steps 2 --warmup 1
