set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r28; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests_full.log 2>&1 || { tail -40 $O/gpu_tests_full.log; exit 1; }
tail -3 $O/gpu_tests_full.log
bash tools/gpu_prof.sh tp8sim_r2 "--simulate-tp 8" > /dev/null && head -20 gpurun_out/rocprof_70b_tp8sim_r2_kernels.txt
bash tools/gpu_prof.sh tp1_b64_r2 "--batch 64" > /dev/null && head -20 gpurun_out/rocprof_70b_tp1_b64_r2_kernels.txt
