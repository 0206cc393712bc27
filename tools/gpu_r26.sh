set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r26; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "oproj" > $O/test_oproj.log 2>&1 || { tail -40 $O/test_oproj.log; exit 1; }
tail -2 $O/test_oproj.log
timeout -k 10 300 python tools/kbench.py --tp 8 > $O/kbench_tp8.txt 2>&1 && grep -E "o_proj|attn" $O/kbench_tp8.txt
timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 5 --warmup 1 --json-out $O/tp8sim.json > $O/tp8sim.log 2>&1 && cat $O/tp8sim.json
