set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r34; mkdir -p $O
timeout -k 10 600 python -u tools/mgemm_tune.py --tp 1 --m 64 --verbose > $O/cands_tp1_m64.txt 2>&1; tail -8 $O/cands_tp1_m64.txt
