set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r22; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampler or nucleus" > $O/test_sampler.log 2>&1 || { tail -30 $O/test_sampler.log; exit 1; }
tail -1 $O/test_sampler.log
timeout -k 10 300 python tools/kbench.py --tp 8 > $O/kbench_tp8.txt 2>&1 && grep sampler $O/kbench_tp8.txt
for R in 2 3; do
timeout -k 10 300 python -u bench.py --arrival-rate $R --steps 40 --warmup 4 --batch 16 --json-out $O/arrival_r$R.json > $O/arrival_r$R.log 2>&1 && cat $O/arrival_r$R.json || exit 1
done
