# Split cost of the two-micro-batch prefill at one TP rank's shapes (collectives skipped), then the multi-rank tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/overlap2; mkdir -p $O
timeout -k 10 400 python -u tools/overlap_probe.py --simulate-tp 8 --layers 20 --reps 3 > $O/split_cost_tp8.jsonl 2> $O/split_cost_tp8.err || { tail -30 $O/split_cost_tp8.err; exit 1; }
cat $O/split_cost_tp8.jsonl
timeout -k 10 400 python -u tools/overlap_probe.py --simulate-tp 2 --layers 10 --reps 3 --sweep 256 2048 8192 > $O/split_cost_tp2.jsonl 2> $O/split_cost_tp2.err || { tail -30 $O/split_cost_tp2.err; exit 1; }
cat $O/split_cost_tp2.jsonl
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_multigpu.py tests/test_prefill_overlap.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "rehearsal|passed|failed" $O/tests.log
