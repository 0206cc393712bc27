# MX plans (keys 3 / 4) for the TP = 2 and TP = 8 shard shapes, which had none (heuristic plans); before / after bench
# rows of one simulated rank at batch 64 on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/mxtp28; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run tp8_fp8_b64_old 600 --simulate-tp 8 --dtype fp8 --batch 64 --steps 3 --warmup 1
run tp2_fp8_b64_old 600 --simulate-tp 2 --dtype fp8 --batch 64 --steps 3 --warmup 1
timeout -k 10 700 python -u tools/mgemm_tune.py --mx --tp 2 8 --m 32 64 128 256 --only qkv o_proj gate_up down --write > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/mgemm_gfx950.json
grep -v cand $O/tune.txt
run tp8_fp8_b64_new 600 --simulate-tp 8 --dtype fp8 --batch 64 --steps 3 --warmup 1
run tp2_fp8_b64_new 600 --simulate-tp 2 --dtype fp8 --batch 64 --steps 3 --warmup 1
