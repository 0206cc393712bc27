set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/kbench.py --tp 8 > gpurun_out/kbench_tp8.txt 2>&1 && cat gpurun_out/kbench_tp8.txt
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_tp1.json 2> gpurun_out/bench_tp1.err && cat gpurun_out/bench_tp1.json
