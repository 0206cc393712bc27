# (Round-5 probe; configs 37-39 were removed again: no gain -- profiles/mgemm_deep_ring_tune_r5.txt.)
# 64-row bf16 QKV / O with deeper LDS rings (mgemm configs 37-39): more weight bytes in flight per CU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/deep; mkdir -p $O
timeout -k 10 600 python -u tools/mgemm_tune.py --tp 1 4 --m 32 64 --only qkv o_proj down --verbose > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v cand $O/tune.txt | tail -20
grep "cfg 3[789]" $O/tune.txt | head -40
