set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r25; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "oproj or split or attention" > $O/test_oproj.log 2>&1 || { tail -40 $O/test_oproj.log; exit 1; }
tail -3 $O/test_oproj.log
timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 5 --warmup 1 --json-out $O/tp8sim.json > $O/tp8sim.log 2>&1 && cat $O/tp8sim.json
K8S_FUSE_ATTN_O=0 timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 5 --warmup 1 --json-out $O/tp8sim_nofuse.json > $O/tp8sim_nofuse.log 2>&1 && cat $O/tp8sim_nofuse.json
