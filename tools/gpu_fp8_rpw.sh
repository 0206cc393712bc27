# A/B: rows per wave of the fp8 decode GEMVs (heuristic vs K8S_GEMV_RPW1=2), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/fp8rpw; mkdir -p $O
run() {
  env $2 timeout -k 10 400 python -u bench.py $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decode_ms_per_step'])" $O/$1.json $1
}
for i in 1 2; do
  run fp8_tp1_default_$i "" "--dtype fp8 --steps 4 --warmup 1"
  run fp8_tp1_rpw2_$i "K8S_GEMV_RPW1=2" "--dtype fp8 --steps 4 --warmup 1"
  run fp8_tp4_default_$i "" "--dtype fp8 --simulate-tp 4 --steps 8 --warmup 2"
  run fp8_tp4_rpw2_$i "K8S_GEMV_RPW1=2" "--dtype fp8 --simulate-tp 4 --steps 8 --warmup 2"
done
