set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r33; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or linear_norm" > $O/test_gemv.log 2>&1 || { tail -30 $O/test_gemv.log; exit 1; }
tail -1 $O/test_gemv.log
for TP in 1 8; do
  timeout -k 10 300 python tools/kbench.py --tp $TP > $O/kb_tp${TP}_nt512.txt 2>&1 && grep -E "norm" $O/kb_tp${TP}_nt512.txt
  K8S_GEMV_NORM_NT=256 timeout -k 10 300 python tools/kbench.py --tp $TP > $O/kb_tp${TP}_nt256.txt 2>&1 && grep -E "norm" $O/kb_tp${TP}_nt256.txt
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $O/tp1.json 2>/dev/null && cat $O/tp1.json
K8S_GEMV_NORM_NT=256 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $O/tp1_nt256.json 2>/dev/null && cat $O/tp1_nt256.json
