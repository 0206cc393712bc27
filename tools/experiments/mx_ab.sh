# K16 MX activations A/B (fp8 weights): MX + model GPU tests, then fp8 bench rows with K8S_MX=1 / 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/mx_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mx_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run fp8_b64_mx 600 K8S_MX=1 --dtype fp8 --batch 64 --steps 3 --warmup 1
run fp8_b64_pt 600 K8S_MX=0 --dtype fp8 --batch 64 --steps 3 --warmup 1
run fp8_tp4_b64_mx 600 K8S_MX=1 --dtype fp8 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run fp8_tp4_b64_pt 600 K8S_MX=0 --dtype fp8 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run fp8_b32_mx 600 K8S_MX=1 --dtype fp8 --batch 32 --steps 3 --warmup 1
run fp8_b32_pt 600 K8S_MX=0 --dtype fp8 --batch 32 --steps 3 --warmup 1
