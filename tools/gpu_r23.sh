set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r23; mkdir -p $O
timeout -k 10 300 python -u bench.py --arrival-rate 2 --steps 30 --warmup 4 --batch 16 --json-out $O/arrival_r2.json > $O/arrival_r2.log 2>&1 && cat $O/arrival_r2.json
