# Refresh the PERF.md bench rows at HEAD (one MI355X).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/matrix; mkdir -p $O
run() {
  timeout -k 10 500 python -u bench.py $2 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['p50_decision_latency_ms'], d['decode_ms_per_step'], d['prefill_ms_per_decision'])" $O/$1.json $1
}
run tp1_b64 "--batch 64 --steps 2 --warmup 1"
run tp8sim_b64 "--batch 64 --steps 3 --warmup 1 --simulate-tp 8"
run tp1_b8 "--batch 8 --steps 3 --warmup 1"
run fp8_tp1 "--dtype fp8 --steps 5 --warmup 1"
run fp8_tp4sim "--dtype fp8 --simulate-tp 4 --steps 10 --warmup 2"
run fp8_tp1_b64 "--dtype fp8 --batch 64 --steps 2 --warmup 1"
run tp1_topp09 "--top-p 0.9 --steps 4 --warmup 1"
run tp1_gen200 "--gen-tokens 200 --steps 3 --warmup 1"
run tp8sim_gen200 "--gen-tokens 200 --simulate-tp 8 --steps 5 --warmup 1"
