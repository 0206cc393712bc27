set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r20; mkdir -p $O
timeout -k 10 400 python -u tools/mgemm_tune.py --tp 1 8 --m 2 4 8 --json-out $O/small_m_bf16.json > $O/small_m_bf16.txt 2>&1 || { tail -20 $O/small_m_bf16.txt; exit 1; }
cat $O/small_m_bf16.txt
timeout -k 10 600 python -u tools/mgemm_tune.py --fp8 --tp 1 4 --m 2 4 8 16 32 48 64 96 128 192 256 --json-out $O/fp8.json > $O/fp8.txt 2>&1 || { tail -20 $O/fp8.txt; exit 1; }
tail -3 $O/fp8.txt
