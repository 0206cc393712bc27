# Prefill all-reduce overlap: multi-rank tests, the split/unsplit probe and a kernel-trace timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
O=$REPO/gpurun_out/overlap; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_multigpu.py tests/test_prefill_overlap.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|SKIP|FAIL|rehearsal" $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "graph or engine" > $O/test_model.log 2>&1 || { tail -30 $O/test_model.log; exit 1; }
tail -1 $O/test_model.log
timeout -k 10 300 python -u tools/overlap_probe.py --world 2 --layers 8 --tokens 256 > $O/probe_w2.json 2> $O/probe_w2.err || { tail -30 $O/probe_w2.err; exit 1; }
cat $O/probe_w2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $REPO/tools/overlap_probe.py --world 2 --layers 4 --tokens 256 --reps 2 --modes split > $O/trace.log 2>&1 || { tail -30 $O/trace.log; exit 1; }
python3 $REPO/tools/overlap_timeline.py $O/trace > $O/timeline.txt && cat $O/timeline.txt
find $O/trace -name "*kernel_trace.csv" | head -4
