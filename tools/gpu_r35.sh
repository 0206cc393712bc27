set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r35; mkdir -p $O
for N in 16 64; do
  timeout -k 10 400 python -u bench.py --nodes $N --steps 3 --warmup 1 --json-out $O/nodes$N.json > $O/nodes$N.log 2>&1 && cat $O/nodes$N.json || exit 1
done
timeout -k 10 600 python -u bench.py --nodes 256 --steps 2 --warmup 1 --max-model-len 32768 --json-out $O/nodes256.json > $O/nodes256.log 2>&1 && cat $O/nodes256.json
