set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r29; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multigpu.py tests/test_mgemm_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/mgemm_fuse_probe.py > $O/fuse_probe.txt 2>&1 && cat $O/fuse_probe.txt
timeout -k 10 300 python -u bench.py --batch 64 --steps 2 --warmup 1 --json-out $O/b64.json > $O/b64.log 2>&1 && cat $O/b64.json
timeout -k 10 300 python -u bench.py --batch 64 --simulate-tp 8 --steps 2 --warmup 1 --json-out $O/b64_tp8sim.json > $O/b64_tp8sim.log 2>&1 && cat $O/b64_tp8sim.json
bash tools/gpu_prof.sh tp8sim_r2 "--simulate-tp 8" > /dev/null && head -16 gpurun_out/rocprof_70b_tp8sim_r2_kernels.txt
bash tools/gpu_prof.sh tp1_b64_r2 "--batch 64" > /dev/null && head -16 gpurun_out/rocprof_70b_tp1_b64_r2_kernels.txt
