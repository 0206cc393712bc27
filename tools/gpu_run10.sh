set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mg10.log 2>&1 || { echo "MGEMM FAILED"; tail -30 gpurun_out/mg10.log; exit 1; }
tail -1 gpurun_out/mg10.log
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/corr_multirank.log 2>&1 || { echo "MULTI-RANK TESTS FAILED"; tail -40 gpurun_out/corr_multirank.log; exit 1; }
grep -E "PASS|FAIL|SKIP|rehearsal" gpurun_out/corr_multirank.log | tail -12
timeout -k 10 400 python -u tools/mgemm_tune.py --tp 1 8 --m 256 512 2048 8192 --json-out gpurun_out/mg_big.json > gpurun_out/mg_big.txt 2>&1 || { tail -20 gpurun_out/mg_big.txt; exit 1; }
cat gpurun_out/mg_big.txt
