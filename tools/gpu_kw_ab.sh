# A/B of the GEMV K-split heuristic (default) against K8S_GEMV_KW=1, interleaved to cancel drift.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/kw_ab; mkdir -p $O
run() {  # tag, env, bench args
  env $2 timeout -k 10 300 python -u bench.py $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decode_ms_per_step'], d['prefill_ms_per_decision'])" $O/$1.json "$1"
}
for i in 1 2; do
  run tp8_default_$i "" "--simulate-tp 8 --steps 15 --warmup 2"
  run tp8_kw1_$i "K8S_GEMV_KW=1" "--simulate-tp 8 --steps 15 --warmup 2"
done
for i in 1 2; do
  run 8b_default_$i "" "--preset llama-3-8b --steps 10 --warmup 2"
  run 8b_kw1_$i "K8S_GEMV_KW=1" "--preset llama-3-8b --steps 10 --warmup 2"
done
run tp1_default "" "--steps 4 --warmup 1"
run tp1_kw1 "K8S_GEMV_KW=1" "--steps 4 --warmup 1"
