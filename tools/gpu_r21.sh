set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r21; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_mgemm_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for B in 4 8; do
  timeout -k 10 300 python -u bench.py --batch $B --steps 2 --warmup 1 --json-out $O/b$B.json > $O/b$B.log 2>&1 && cat $O/b$B.json || exit 1
done
timeout -k 10 300 python -u bench.py --batch 8 --simulate-tp 8 --steps 2 --warmup 1 --json-out $O/b8_tp8sim.json > $O/b8_tp8sim.log 2>&1 && cat $O/b8_tp8sim.json
timeout -k 10 300 python -u bench.py --arrival-rate 3 --steps 40 --warmup 4 --batch 16 --json-out $O/arrival.json > $O/arrival.log 2>&1 && cat $O/arrival.json
timeout -k 10 300 python -u bench.py --gen-tokens 200 --steps 3 --warmup 1 --json-out $O/g200_tp1.json > $O/g200_tp1.log 2>&1 && cat $O/g200_tp1.json
timeout -k 10 300 python -u bench.py --gen-tokens 200 --simulate-tp 8 --steps 5 --warmup 1 --json-out $O/g200_tp8sim.json > $O/g200_tp8sim.log 2>&1 && cat $O/g200_tp8sim.json
