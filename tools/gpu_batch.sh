# 1-GPU batched benches (BASELINE config 4): 64 pods per step, reference layout and cluster_first; fp8 too.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "ref:--prompt-layout reference" "cf:--prompt-layout cluster_first" "fp8:--dtype fp8"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --batch 64 $args > gpurun_out/bench_b64_$tag.json 2> gpurun_out/bench_b64_$tag.err || { tail -20 gpurun_out/bench_b64_$tag.err; exit 1; }
  cat gpurun_out/bench_b64_$tag.json
done
