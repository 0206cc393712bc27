# Split decode attention after a kernel change: its tests, the per-kernel microbench, the TP=8-shape decode bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn or decode" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/kbench.py --tp 8 > $O/kbench_tp8.txt 2>&1 && grep -E "decode_attn\[split\]" $O/kbench_tp8.txt
timeout -k 10 300 python tools/kbench.py --tp 1 > $O/kbench_tp1.txt 2>&1 && grep -E "decode_attn\[split\]" $O/kbench_tp1.txt
timeout -k 10 600 python -u bench.py --simulate-tp 8 --steps 10 --warmup 2 > $O/bench_tp8sim.json 2> $O/bench_tp8sim.err || { tail -20 $O/bench_tp8sim.err; exit 1; }
cat $O/bench_tp8sim.json
