set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r36; mkdir -p $O
timeout -k 10 400 python -u bench.py --nodes 64 --max-model-len 8192 --steps 3 --warmup 1 --json-out $O/nodes64.json > $O/nodes64.log 2>&1 && cat $O/nodes64.json
timeout -k 10 400 python -u bench.py --nodes 256 --max-model-len 32768 --simulate-tp 8 --steps 2 --warmup 1 --json-out $O/nodes256_tp8sim.json > $O/nodes256_tp8sim.log 2>&1 && cat $O/nodes256_tp8sim.json
