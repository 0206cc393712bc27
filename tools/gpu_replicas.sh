# Engine replicas (data parallelism) on one GPU, then smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/replicas; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_replicas_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "replicas|PASS|FAIL|passed" $O/tests.log
K8S_SMOKE=1 timeout -k 10 300 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
