# decision rate / latency vs cluster size (3, 16, 64, 256 nodes) on 70B TP=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for n in ${NODES:-16 64 256}; do
  timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --nodes $n --max-model-len ${MAXLEN:-32768} > gpurun_out/bench_nodes_$n.json 2> gpurun_out/bench_nodes_$n.err || { tail -20 gpurun_out/bench_nodes_$n.err; exit 1; }
  cat gpurun_out/bench_nodes_$n.json
done
