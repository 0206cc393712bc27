# Kernel + multi-rank correctness on one GPU: mgemm, the kernel suite (GQA prefill attention), the
# 8/4-rank rehearsal and the xGMI fault path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mgemm_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/corr_kernels.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -40 gpurun_out/corr_kernels.log; exit 1; }
tail -2 gpurun_out/corr_kernels.log
timeout -k 10 600 python -u -m pytest tests/test_faults_gpu.py tests/test_multigpu.py tests/test_xgmi_gpu.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/corr_multirank.log 2>&1 || { echo "MULTI-RANK TESTS FAILED"; tail -60 gpurun_out/corr_multirank.log; exit 1; }
grep -E "PASS|FAIL|SKIP|rehearsal|xgmi all-reduce" gpurun_out/corr_multirank.log | tail -20
