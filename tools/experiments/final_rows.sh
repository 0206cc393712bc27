# One row per configuration for docs/PERF.md (round 5 close): each bench in its own time limit, JSON lines collected.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/final; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run nodes16 300 --nodes 16 --steps 10 --warmup 2
run nodes64 400 --nodes 64 --max-model-len 8192 --steps 10 --warmup 2
run llama8b 300 --preset llama-3-8b --steps 10 --warmup 2
run tp8sim 300 --simulate-tp 8 --steps 10 --warmup 2
run tp4sim 300 --simulate-tp 4 --steps 10 --warmup 2
run tp2sim 300 --simulate-tp 2 --steps 10 --warmup 2
run fp8 300 --dtype fp8 --steps 10 --warmup 2
run fp8_tp4sim 300 --dtype fp8 --simulate-tp 4 --steps 10 --warmup 2
run b8 300 --batch 8 --steps 10 --warmup 2
run b64 600 --batch 64 --steps 3 --warmup 1
run tp8sim_b64 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
