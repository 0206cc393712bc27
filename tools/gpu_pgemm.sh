# pgemm.hip: numerics tests, then the prefill-shape tuning sweep vs the library GEMM and mgemm.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pgemm_gpu.py -x -v --timeout 120 --timeout-method thread ${PG_TEST_ARGS:-} > gpurun_out/pgemm_tests.log 2>&1 || { echo "PGEMM TESTS FAILED"; tail -60 gpurun_out/pgemm_tests.log; exit 1; }
tail -3 gpurun_out/pgemm_tests.log
timeout -k 10 ${TUNE_TIMEOUT:-500} python -u tools/pgemm_tune.py ${TUNE_ARGS:---tp 1 --m 256 2048} --json-out gpurun_out/pgemm_tune.json > gpurun_out/pgemm_tune.txt 2>&1 || { tail -30 gpurun_out/pgemm_tune.txt; exit 1; }
cat gpurun_out/pgemm_tune.txt
