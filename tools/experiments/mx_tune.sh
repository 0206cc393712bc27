# MX tests, re-tune gate/up's MX-output plans (TP = 1 / 4, 32-256 rows), then the fp8 batch-64 / batch-1 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mx_gpu.py > gpurun_out/mx_tests.log 2>&1 || { tail -30 gpurun_out/mx_tests.log; exit 1; }
tail -1 gpurun_out/mx_tests.log
timeout -k 10 600 python -u tools/mgemm_tune.py --mx --tp 1 4 --m 32 64 128 256 --only gate_up --write --verbose > gpurun_out/mx_tune_gu.txt 2>&1 || exit 1
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json gpurun_out/mgemm_gfx950.json
grep -v cand gpurun_out/mx_tune_gu.txt | tail -12
O=gpurun_out/mx_ab; mkdir -p $O
run() {  # run <label> <seconds> <env> <bench args...>
  local label=$1 t=$2 e=$3; shift 3
  env $e timeout -k 10 "$t" python -u bench.py "$@" > "$O/$label.json" 2> "$O/$label.err" || { echo "$label FAILED"; tail -5 "$O/$label.err"; exit 1; }
  echo "$label $(tail -1 $O/$label.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"], d.get("prefill_ms_per_decision"))')"
}
run fp8_b64_mx 600 K8S_MX=1 --dtype fp8 --batch 64 --steps 3 --warmup 1
run fp8_b64_pt 600 K8S_MX=0 --dtype fp8 --batch 64 --steps 3 --warmup 1
run fp8_tp4_b64_mx 600 K8S_MX=1 --dtype fp8 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
run fp8_tp4_b64_pt 600 K8S_MX=0 --dtype fp8 --simulate-tp 4 --batch 64 --steps 3 --warmup 1
