# Multi-rank rehearsal (8 and 4 ranks on one GPU) incl. speculative decoding at TP = 8, and the speculative tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/mr; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_multigpu.py tests/test_speculative_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "rehearsal|PASS|FAIL|passed" $O/tests.log
