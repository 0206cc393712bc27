# --simulate-tp 8 decode A/B of the GEMV knobs (one bench each, same box): K8S_GEMV_KW, K8S_GEMV_RPW1, K8S_GEMV_LOOP.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/tp8ab; mkdir -p $O
for v in base K8S_GEMV_KW=2 K8S_GEMV_RPW1=2 K8S_GEMV_LOOP=2 base; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env $e timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 6 --warmup 2 > "$O/b_${v%%=*}.json" 2>&1 || exit 1
  echo "$v $(tail -1 $O/b_${v%%=*}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"])')"
done
