# 8B decode kernel profile, then GEMV launch knobs at one TP=8 rank's shapes (decode ms/token).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/knobs; mkdir -p $O
bash tools/gpu_prof.sh 8b "--preset llama-3-8b" > $O/prof8b.txt 2>&1 || { tail -20 $O/prof8b.txt; exit 1; }
head -24 $O/prof8b.txt
for kv in "" "K8S_GEMV_KW=1" "K8S_GEMV_RPW1=2"; do
  env $kv timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 6 --warmup 2 > $O/tp8_$kv.json 2> $O/tp8_$kv.err || { tail -20 $O/tp8_$kv.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2] or 'default', d['value'], d['decode_ms_per_step'], d['prefill_ms_per_decision'])" $O/tp8_$kv.json "$kv"
done
