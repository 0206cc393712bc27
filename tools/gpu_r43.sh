set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r43; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or model or decode" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u bench.py --batch 64 --simulate-tp 8 --steps 2 --warmup 1 --json-out $O/b64_tp8sim.json > $O/b64_tp8sim.log 2>&1 && cat $O/b64_tp8sim.json
timeout -k 10 300 python -u bench.py --batch 8 --steps 2 --warmup 1 --json-out $O/b8.json > $O/b8.log 2>&1 && cat $O/b8.json
timeout -k 10 300 python -u bench.py --batch 16 --simulate-tp 8 --steps 2 --warmup 1 --json-out $O/b16_tp8sim.json > $O/b16_tp8sim.log 2>&1 && cat $O/b16_tp8sim.json
