set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mgemm_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r14_kernels.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -40 gpurun_out/r14_kernels.log; exit 1; }
tail -2 gpurun_out/r14_kernels.log
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py tests/test_xgmi_gpu.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/r14_multi.log 2>&1 || { echo "MULTI TESTS FAILED"; tail -40 gpurun_out/r14_multi.log; exit 1; }
grep -E "rehearsal|passed|failed" gpurun_out/r14_multi.log | tail -4
mkdir -p gpurun_out/b3
run() { tag=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/b3/$tag.json 2> gpurun_out/b3/$tag.err || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/b3/$tag.err; return 1; }; cat gpurun_out/b3/$tag.json; }
run tp1_b64 --steps 2 --warmup 1 --batch 64 && run tp8sim_b64 --steps 2 --warmup 1 --batch 64 --simulate-tp 8 && run tp1 --steps 6 --warmup 2
