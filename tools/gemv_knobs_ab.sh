set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemv_ab
for cfg in "base" "K8S_GEMV_LOOP_MIN_MI=64" "K8S_GEMV_LOOP_BF16=3" "K8S_GEMV_LOOP_BF16=1" "base"; do
  if [ "$cfg" = base ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 > gpurun_out/gemv_ab/out.json 2> gpurun_out/gemv_ab/err.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/gemv_ab/out.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['decode_ms_per_step'], d['prefill_ms_per_decision'])" | tee -a gpurun_out/gemv_ab/summary.txt
done
