set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r30; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py --batch 64 --steps 2 --warmup 1 --json-out $O/b64.json > $O/b64.log 2>&1 && cat $O/b64.json
timeout -k 10 300 python -u bench.py --batch 16 --steps 2 --warmup 1 --json-out $O/b16.json > $O/b16.log 2>&1 && cat $O/b16.json
timeout -k 10 300 python -u bench.py --batch 64 --dtype fp8 --steps 2 --warmup 1 --json-out $O/b64_fp8.json > $O/b64_fp8.log 2>&1 && cat $O/b64_fp8.json
timeout -k 10 300 python -u bench.py --dtype fp8 --steps 3 --warmup 1 --json-out $O/fp8.json > $O/fp8.log 2>&1 && cat $O/fp8.json
timeout -k 10 300 python -u bench.py --preset llama-3-8b --steps 5 --warmup 1 --json-out $O/8b.json > $O/8b.log 2>&1 && cat $O/8b.json
