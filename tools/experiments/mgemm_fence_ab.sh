# mgemm split tiles: write-through slab stores + relaxed ticket (K8S_MGEMM_FENCED=0; tests run in that mode) vs
# (K8S_MGEMM_FENCED=1, the round-4 form).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/fence; mkdir -p $O
K8S_MGEMM_FENCED=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mgemm_gpu.py tests/test_mx_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run tp8_b64_coherent 600 K8S_MGEMM_FENCED=0 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run tp8_b64_fenced 600 "" --simulate-tp 8 --batch 64 --steps 3 --warmup 1
run b64_coherent 600 K8S_MGEMM_FENCED=0 --batch 64 --steps 3 --warmup 1
run b64_fenced 600 "" --batch 64 --steps 3 --warmup 1
run fp8_b64_coherent 600 K8S_MGEMM_FENCED=0 --dtype fp8 --batch 64 --steps 3 --warmup 1
run fp8_b64_fenced 600 "" --dtype fp8 --batch 64 --steps 3 --warmup 1
run tp8_b64_coherent2 600 K8S_MGEMM_FENCED=0 --simulate-tp 8 --batch 64 --steps 3 --warmup 1
