# 8-row decode A/B: per-layer kernel view of the default, then decode-attention partition 512
# and two sgemv workgroups per CU, one bench each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/b8; mkdir -p $O
mkdir -p gpurun_out/mfma && hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_shape_probe tools/experiments/mfma_shape_probe.hip && timeout -k 10 60 /tmp/mfma_shape_probe 4096 > gpurun_out/mfma/probe.txt && cat gpurun_out/mfma/probe.txt || exit 1
bash tools/gpu_prof.sh tp1_b8 "--batch 8" > /dev/null && cat gpurun_out/lastfwd_tp1_b8.txt || exit 1
bash tools/gpu_prof.sh tp1_b1 "" > /dev/null && cat gpurun_out/lastfwd_tp1_b1.txt || exit 1
for v in "base" "K8S_ATTN_FUSED_PART=512" "K8S_SGEMV_WG_PER_CU=2"; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env $e timeout -k 10 400 python -u bench.py --batch 8 --steps 10 --warmup 2 > "$O/b8_${v%%=*}.json" 2>&1 || exit 1
  echo "$v $(tail -1 $O/b8_${v%%=*}.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_ms_per_step"])')"
done
