set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r42; mkdir -p $O
for M in 4 8 16 32 64; do
  timeout -k 10 300 python tools/kbench.py --tp 1 --M $M > $O/kb_tp1_M$M.txt 2>&1 && echo "== TP1 M=$M" && grep -E "decode_attn.*ctx=564 maxctx=1024" $O/kb_tp1_M$M.txt
done
for M in 32 64; do
  timeout -k 10 300 python tools/kbench.py --tp 8 --M $M > $O/kb_tp8_M$M.txt 2>&1 && echo "== TP8 M=$M" && grep -E "decode_attn.*ctx=564 maxctx=1024" $O/kb_tp8_M$M.txt
done
