# Quick GPU iteration: selected GPU tests (pytest -k expression in $1) + TP=8-shape kernel microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${1:-.}" > gpurun_out/gpu_quick_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/gpu_quick_tests.log; exit 1; }
tail -2 gpurun_out/gpu_quick_tests.log
timeout -k 10 300 python tools/kbench.py --tp "${2:-8}" > gpurun_out/kbench.txt 2>&1 && cat gpurun_out/kbench.txt
