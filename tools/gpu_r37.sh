set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r37; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemv or linear_norm or model or decode" > $O/test_gemv.log 2>&1 || { tail -30 $O/test_gemv.log; exit 1; }
tail -1 $O/test_gemv.log
for TP in 8 1; do
  timeout -k 10 300 python tools/kbench.py --tp $TP > $O/kb_tp${TP}.txt 2>&1 && grep -E "qkv|gate_up|lm_head" $O/kb_tp${TP}.txt
done
timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 5 --warmup 1 > $O/tp8sim.json 2>/dev/null && cat $O/tp8sim.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $O/tp1.json 2>/dev/null && cat $O/tp1.json
