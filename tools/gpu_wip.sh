set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wip_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/wip_tests.log; exit 1; }
tail -3 gpurun_out/wip_tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --simulate-tp 8 > gpurun_out/bench_tp8sim.json 2> gpurun_out/bench_tp8sim.err || { tail -20 gpurun_out/bench_tp8sim.err; exit 1; }
cat gpurun_out/bench_tp8sim.json
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_tp1.json 2> gpurun_out/bench_tp1.err || { tail -20 gpurun_out/bench_tp1.err; exit 1; }
cat gpurun_out/bench_tp1.json
