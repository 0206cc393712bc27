# QKV plans re-tuned with the RMS prologue on (as the decode layer runs them: TP = 2 / 4 / 8 at 32-64 rows, every TP
# at 128 rows); before / after bench rows on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/qkvtune; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run tp8_b64_old 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run tp4_b64_old 600 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run b96_old 600 --batch 96 --steps 2 --warmup 1
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --qkv-rms --tp 2 4 8 --m 32 64 --only qkv --write > $O/tune_a.txt 2>&1 || { tail -20 $O/tune_a.txt; exit 1; }
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --qkv-rms --tp 1 2 4 8 --m 128 --only qkv --write > $O/tune_b.txt 2>&1 || { tail -20 $O/tune_b.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/mgemm_gfx950.json
cat $O/tune_a.txt $O/tune_b.txt | grep -v cand
run tp8_b64_new 600 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run tp4_b64_new 600 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run b96_new 600 --batch 96 --steps 2 --warmup 1
