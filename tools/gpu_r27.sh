set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r27; mkdir -p $O
timeout -k 10 300 python tools/kbench.py --tp 8 > $O/kbench_tp8.txt 2>&1 && grep -E "o_proj|split\] ctx=564" $O/kbench_tp8.txt
