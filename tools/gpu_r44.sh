set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r44; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or model or decode" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for M in 32 64; do
  timeout -k 10 300 python tools/kbench.py --tp 1 --M $M > $O/kb_tp1_M$M.txt 2>&1 && echo "== TP1 M=$M" && grep -E "decode_attn\[one-wg\]" $O/kb_tp1_M$M.txt
done
timeout -k 10 300 python -u bench.py --batch 64 --steps 2 --warmup 1 --json-out $O/b64.json > $O/b64.log 2>&1 && cat $O/b64.json
timeout -k 10 300 python -u bench.py --batch 32 --steps 2 --warmup 1 --json-out $O/b32.json > $O/b32.log 2>&1 && cat $O/b32.json
