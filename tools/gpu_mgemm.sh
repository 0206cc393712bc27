# mgemm.hip: numerics tests, then the per-shape tuning sweep vs the library GEMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mgemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mgemm_tests.log 2>&1 || { echo "MGEMM TESTS FAILED"; tail -40 gpurun_out/mgemm_tests.log; exit 1; }
tail -3 gpurun_out/mgemm_tests.log
timeout -k 10 600 python -u tools/mgemm_tune.py ${TUNE_ARGS:---tp 8 1 --m 16 32 64 128 256 512} --json-out gpurun_out/mgemm_tune.json > gpurun_out/mgemm_tune.txt 2>&1 || { tail -20 gpurun_out/mgemm_tune.txt; exit 1; }
cat gpurun_out/mgemm_tune.txt
