# TP=1 17-64-row QKV: separate RMSNorm + plain GEMM (default) vs mgemm's RMS prologue (x.x^T MFMA) with plans tuned
# in situ for it (K8S_RMS_UNFUSED_MIN_N=16384 routes the 10240-feature QKV onto the prologue). One box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/qkvrms; mkdir -p $O
run() {  # run <label> <seconds> <bench args...>
  local label=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run b64_sep 600 --batch 64 --steps 3 --warmup 1
run b32_sep 600 --batch 32 --steps 3 --warmup 1
timeout -k 10 600 python -u tools/mgemm_tune.py --insitu --qkv-rms --tp 1 --m 32 64 --only qkv --json-out $O/tune.json > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v cand $O/tune.txt
export K8S_MGEMM_OVERRIDE=$(python3 -c "import json; r=json.load(open('$O/tune.json')); print(';'.join(f\"{x['M']},{x['N']},{x['K']},{x['epi']},0={x['cfg']}:{x['grid']}\" for x in r))")
echo "override $K8S_MGEMM_OVERRIDE"
export K8S_RMS_UNFUSED_MIN_N=16384
run b64_pro 600 --batch 64 --steps 3 --warmup 1
run b32_pro 600 --batch 32 --steps 3 --warmup 1
