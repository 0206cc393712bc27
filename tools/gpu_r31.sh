set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r31; mkdir -p $O
timeout -k 10 300 python -u bench.py --batch 64 --steps 2 --warmup 1 --json-out $O/b64.json > $O/b64.log 2>&1 && cat $O/b64.json
timeout -k 10 300 python -u bench.py --batch 64 --dtype fp8 --steps 2 --warmup 1 --json-out $O/b64_fp8.json > $O/b64_fp8.log 2>&1 && cat $O/b64_fp8.json
timeout -k 10 300 python -u bench.py --dtype fp8 --simulate-tp 4 --steps 3 --warmup 1 --json-out $O/fp8_tp4sim.json > $O/fp8_tp4sim.log 2>&1 && cat $O/fp8_tp4sim.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --json-out $O/tp1.json > $O/tp1.log 2>&1 && cat $O/tp1.json
